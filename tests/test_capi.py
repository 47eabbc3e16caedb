"""The C-ABI library loads and exports exactly what include/itrails_hip.h declares.
CPU-only: no call here touches a device."""
import ctypes

import pytest

from itrails_amd import _lib


def test_library_exports_every_header_symbol():
    L = _lib.lib()
    syms = _lib.header_symbols()
    assert len(syms) >= 15
    for s in syms:
        assert hasattr(L, s), s
    assert set(syms) == set(_lib._SIGNATURES), "ctypes signatures out of sync with header"


def test_version_and_argument_errors():
    L = _lib.lib()
    assert L.itr_version() == 1
    h = ctypes.c_void_p()
    rc = L.itr_model_create(0, None, None, None, None, None, None, ctypes.byref(h))
    assert rc == _lib.ITR_EINVAL and b"n_states" in L.itr_last_error()
    with pytest.raises(_lib.ItrError):
        _lib.check(L.itr_model_create(500, None, None, None, None, None, None, ctypes.byref(h)))
    rc = L.itr_plan_create(None, -1, ctypes.byref(h))
    assert rc == _lib.ITR_EINVAL
    rc = L.itr_expm_batched(0, 1, None, None, None)
    assert rc == _lib.ITR_EINVAL


def test_plan_rejects_decreasing_offsets():
    import numpy as np

    L = _lib.lib()
    off = np.array([0, 5, 3], dtype=np.int64)
    h = ctypes.c_void_p()
    assert L.itr_plan_create(off.ctypes.data, 2, ctypes.byref(h)) == _lib.ITR_EINVAL
    assert b"decrease" in L.itr_last_error()
