"""ctypes binding of libitrails_hip.so (the C ABI of include/itrails_hip.h).

The shared library is built in-tree by __graft_entry__.build() (or `python -m
itrails_amd.build`).  There is no fallback: if the library is missing or cannot be loaded,
every entry point raises, so a GPU run can never silently use host code.
"""
from __future__ import annotations

import atexit
import ctypes
import os
import re

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("ITR_LIB") or os.path.join(HERE, "libitrails_hip.so")
HEADER = os.path.join(os.path.dirname(HERE), "include", "itrails_hip.h")

ITR_OK, ITR_EINVAL, ITR_EHIP, ITR_ESTATE, ITR_EDATA = 0, 1, 2, 3, 4
NOBS = 625
MAX_STATES = 192

_lib = None

_P = ctypes.c_void_p
_I = ctypes.c_int
_I64 = ctypes.c_int64
_D = ctypes.c_double

_SIGNATURES = {
    "itr_version": ([], _I),
    "itr_last_error": ([], ctypes.c_char_p),
    "itr_device_count": ([ctypes.POINTER(_I)], _I),
    "itr_model_create": ([_I, _P, _P, _P, _P, _P, _P, ctypes.POINTER(_P)], _I),
    "itr_model_destroy": ([_P], _I),
    "itr_model_prepare_viterbi": ([_P], _I),
    "itr_model_n_states": ([_P, ctypes.POINTER(_I)], _I),
    "itr_plan_create": ([_P, _I64, ctypes.POINTER(_P)], _I),
    "itr_plan_create_ex": ([_P, _I64, _D, _D, ctypes.POINTER(_P)], _I),
    "itr_plan_destroy": ([_P], _I),
    "itr_plan_partition_info": ([_P, _I64, _I, _P], _I),
    "itr_plan_set_prune_len": ([_P, _I64], _I),
    "itr_plan_total_columns": ([_P, ctypes.POINTER(_I64)], _I),
    "itr_plan_reserve": ([_P, _I, _I], _I),
    "itr_forward_loglik": ([_P, _P, _P, _P, _P], _I),
    "itr_viterbi": ([_P, _P, _P, _P, _P], _I),
    "itr_forward_viterbi": ([_P, _P, _P, _P, _P, _P], _I),
    "itr_posterior": ([_P, _P, _P, _P, _P], _I),
    "itr_block_rows": ([_P, _I, _P, _I64, _P, _P, _P], _I),
    "itr_backtrack_rows": ([_P, _P, _I64, _I, _P, _P], _I),
    "itr_pack_symbols": ([_P, _P, _I64, _P, _P], _I),
    "itr_forward_loglik_host": ([_P, _P, _P, _P], _I),
    "itr_viterbi_host": ([_P, _P, _P, _P], _I),
    "itr_posterior_host": ([_P, _P, _P, _P], _I),
    "itr_forward_loglik_blocks": ([_P, _P, _P, _P, _I64, _P], _I),
    "itr_viterbi_blocks": ([_P, _P, _P, _P, _I64, _P], _I),
    "itr_release_staging": ([], _I),
    "itr_release_streams": ([], _I),
    "itr_last_kernel_ms": ([ctypes.c_char_p, ctypes.POINTER(_D)], _I),
    "itr_expm_batched": ([_I, _I64, _P, _P, _P], _I),
    "itr_expm_batched_host": ([_I, _I64, _P, _P], _I),
    "itr_expm_blocktri_batched": ([_I, _I, _I64, _P, _P, _P], _I),
    "itr_vanloan_paths": ([_I, _P, _I, _P, _I, _P, _I64, _P, _P, _P, _P, _P], _I),
    "itr_vanloan_paths_ex": ([_I, _P, _I, _P, _I, _P, _I64, _P, _P, _P, _P, _P, _P], _I),
    "itr_vanloan_job_norms": ([_I, _P, _I, _P, _I, _P, _I64, _P, _P, _P, _P], _I),
    "itr_solve_batched": ([_I, _I, _I64, _P, _P, _P], _I),
    "itr_inverse_batched": ([_I, _I64, _P, _P, _P], _I),
    "itr_gemm_batched": ([_I, _I, _I, _I64, _D, _P, _P, _D, _P, _P], _I),
    "itr_chain_rows": ([_I, _I, _I, _P, _P, _P, _P, _P, _P, _I64, _P, _I64, _P, _P, _I64, _P],
                       _I),
    "itr_group_sum": ([_I64, _I, _P, _P, _P, _P, _P], _I),
    "itr_emission_rows": ([_I, _P, _P, _P], _I),
    "itr_maf_open": ([ctypes.c_char_p, ctypes.POINTER(ctypes.c_char_p), ctypes.c_char_p,
                      ctypes.POINTER(_P)], _I),
    "itr_maf_sizes": ([_P, ctypes.POINTER(_I64), ctypes.POINTER(_I64), ctypes.POINTER(_I64),
                       ctypes.POINTER(_I64)], _I),
    "itr_maf_copy": ([_P, _P, _P, _P, _P], _I),
    "itr_maf_close": ([_P], _I),
    "itr_write_viterbi_csv": ([ctypes.c_char_p, _P, _P, _I64, _P, _I64], _I),
    "itr_write_posterior_csv": ([ctypes.c_char_p, _P, _I, _P, _I64, _P, _I64, _I], _I),
    "itr_format_float": ([_D, ctypes.c_char_p, _I], _I),
}


class ItrError(RuntimeError):
    """A non-zero return code from the C ABI."""

    def __init__(self, code: int, msg: str):
        super().__init__(f"itrails_hip error {code}: {msg}")
        self.code = code


def header_symbols() -> list:
    """Entry points declared in include/itrails_hip.h (ITR_API ... name(...))."""
    text = open(HEADER).read()
    return re.findall(r"ITR_API\s+[\w\s\*]+?\b(itr_\w+)\s*\(", text)


def lib():
    """Load the library (once).  Raises ImportError if it was not built."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"{LIB_PATH} is missing: build the HIP extension first "
            "(python -c 'import __graft_entry__ as g; g.build()')")
    # One HIP runtime per process: torch (device memory, streams) is loaded first, so the
    # library's libamdhip64.so.7 resolves to the runtime torch already mapped.  Loaded the
    # other way round, /opt/rocm's runtime and torch's bundled one both open the device and
    # the second reports "no ROCm-capable device".
    import torch  # noqa: F401
    L = ctypes.CDLL(LIB_PATH)
    for name, (args, res) in _SIGNATURES.items():
        if os.environ.get("ITR_LIB") and not hasattr(L, name):
            continue  # (an older library under A/B test: entry points it predates stay unbound)
        f = getattr(L, name)
        f.argtypes = args
        f.restype = res
    _lib = L
    # the CU-masked streams of itr_viterbi go before the HIP runtime is torn down
    atexit.register(L.itr_release_streams)
    return L


def check(rc: int) -> None:
    if rc != ITR_OK:
        msg = lib().itr_last_error()
        raise ItrError(rc, msg.decode() if msg else "")


def ptr(x) -> int:
    """Device or host address of a torch tensor / numpy array (or a raw int)."""
    if x is None:
        return None
    if isinstance(x, int):
        return x
    if hasattr(x, "data_ptr"):
        return x.data_ptr()
    return x.ctypes.data
