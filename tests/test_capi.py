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


def test_one_hip_runtime_when_library_loads_first():
    """Loading the library before anything imports torch must not map a second HIP runtime
    next to torch's (two runtimes in one process: the second finds no device)."""
    import subprocess
    import sys
    code = ("import itrails_amd._lib as L; L.lib(); import torch; "
            "m = open('/proc/self/maps').read(); "
            "print(len({l.split()[-1] for l in m.splitlines() if 'libamdhip64' in l}))")
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True,
                         check=True, cwd=_lib.os.path.dirname(_lib.HERE))
    assert out.stdout.strip().splitlines()[-1] == "1"


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


def test_pack_symbols_matches_numpy_and_rejects_bad_symbols():
    """itr_pack_symbols (host only) == the NumPy concatenation; out-of-alphabet symbols
    raise IndexError like the reference's fancy index; empty and ragged blocks."""
    import numpy as np

    from itrails_amd import hmm

    rng = np.random.default_rng(5)
    lens = [0, 1, 7, 0, 3000, 1 << 20, 2, 0]  # enough columns for several threads
    V = [rng.integers(0, 625, n).astype(np.int64) for n in lens]
    obs, off = hmm.concat_blocks(V)
    assert obs.dtype == np.uint16 and off.dtype == np.int64
    assert np.array_equal(off, np.concatenate([[0], np.cumsum(lens)]))
    assert np.array_equal(obs, np.concatenate(V).astype(np.uint16))
    # non-int64 input takes the NumPy path and agrees
    o2, f2 = hmm.concat_blocks([v.astype(np.int32) for v in V])
    assert np.array_equal(o2, obs) and np.array_equal(f2, off)
    for bad in (625, -1, 1 << 40):
        W = [v.copy() for v in V]
        W[5][12345] = bad
        with pytest.raises(IndexError, match="block 5, column 12345"):
            hmm.concat_blocks(W)
    e, eo = hmm.concat_blocks([np.zeros(0, dtype=np.int64)] * 3)
    assert e.size == 0 and np.array_equal(eo, [0, 0, 0, 0])


def test_vlst_scan_extension():
    """The V_lst scan of the host-block entry points (csrc/blocks_ext.c): lengths and data
    pointers of 1-D C-contiguous int64 arrays; anything else (other dtypes, 2-D, strided,
    byte-swapped, lists) takes the NumPy packing path (None)."""
    import numpy as np

    from itrails_amd import hmm

    assert hmm._blocks_ext is not None  # built with the library (itrails_amd/build.py)
    V = [np.arange(k % 37, dtype=np.int64) for k in range(3000)]
    lens, ptrs, off = hmm._lens_ptrs(V)
    assert np.array_equal(lens, [len(v) for v in V])
    assert np.array_equal(ptrs, [v.ctypes.data for v in V])
    assert np.array_equal(off, np.concatenate([[0], np.cumsum(lens)]))
    for bad in (np.zeros(3, np.int32), np.zeros((2, 2), np.int64), np.zeros(6, np.int64)[::2],
                np.zeros(3, ">i8"), [1, 2]):
        assert hmm._lens_ptrs(V[:5] + [bad]) is None
