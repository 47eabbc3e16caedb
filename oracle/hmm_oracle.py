"""ctypes binding of oracle/hmm_oracle.c — TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

Each function mirrors the reference function it restates (optimizer.py:145-354) and takes
the same per-symbol tables the device path consumes (itrails_amd/tables.py).
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# (ITR_ORACLE_LIB: another build of the same source, e.g. the sanitizer build of
# scripts/asan_host.sh)
LIB = os.environ.get("ITR_ORACLE_LIB") or os.path.join(HERE, "liboracle.so")

_lib = None


def build(force: bool = False) -> str:
    src = os.path.join(HERE, "hmm_oracle.c")
    if os.environ.get("ITR_ORACLE_LIB"):
        return LIB
    if force or not os.path.exists(LIB) or os.path.getmtime(LIB) < os.path.getmtime(src):
        subprocess.run(["make", "-s", "-C", HERE, "liboracle.so"], check=True)
    return LIB


def lib():
    global _lib
    if _lib is None:
        build()
        L = ctypes.CDLL(LIB)
        P = ctypes.c_void_p
        L.oracle_forward_loglik.argtypes = [ctypes.c_int, P, P, P, P, P, ctypes.c_int64, P]
        L.oracle_viterbi.argtypes = [ctypes.c_int, P, P, P, P, P, ctypes.c_int64, P]
        L.oracle_posterior.argtypes = [ctypes.c_int, P, P, P, P, P, ctypes.c_int64, P]
        L.oracle_set_threads.argtypes = [ctypes.c_int]
        for f in (L.oracle_forward_loglik, L.oracle_viterbi, L.oracle_posterior,
                  L.oracle_set_threads):
            f.restype = None
        _lib = L
    return _lib


def set_threads(k: int) -> None:
    """OpenMP threads of the following calls."""
    lib().oracle_set_threads(int(k))


def _p(x):
    return x.ctypes.data_as(ctypes.c_void_p)


def _prep(obs, off):
    obs = np.ascontiguousarray(obs, dtype=np.uint16)
    off = np.ascontiguousarray(off, dtype=np.int64)
    return obs, off


def forward_loglik(tables, obs, off) -> np.ndarray:
    obs, off = _prep(obs, off)
    out = np.zeros(len(off) - 1)
    lib().oracle_forward_loglik(tables.n, _p(tables.a), _p(tables.emit), _p(tables.pi_emit),
                                _p(obs), _p(off), len(off) - 1, _p(out))
    return out


def viterbi(tables, obs, off) -> np.ndarray:
    obs, off = _prep(obs, off)
    out = np.zeros(int(off[-1]), dtype=np.int16)
    lib().oracle_viterbi(tables.n, _p(tables.log_a), _p(tables.log_emit),
                         _p(tables.log_pi_emit), _p(obs), _p(off), len(off) - 1, _p(out))
    return out


def posterior(tables, obs, off) -> np.ndarray:
    obs, off = _prep(obs, off)
    out = np.zeros((int(off[-1]), tables.n))
    lib().oracle_posterior(tables.n, _p(tables.a), _p(tables.emit), _p(tables.pi_emit),
                           _p(obs), _p(off), len(off) - 1, _p(out))
    return out
