"""Per-column HMM tables the device sweeps consume, built on the host with NumPy.

The reference re-evaluates, for every column t of every block, the emission vector
`b[:, order[V[t]]].sum(axis=1)` and, in Viterbi, `np.log(a)` and `np.log(e)`
(optimizer.py:182, 186, 210, 323, 328-329).  These depend only on the symbol (625 of them),
so they are tabulated once per model with the very same NumPy expressions, row by row.
Identical inputs to identical NumPy calls give bit-identical tables, which is what makes the
device Viterbi path bit-exact against the reference.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

from .read_data import NOBS, get_idx_state


@dataclass(frozen=True)
class HmmTables:
    n: int
    a: np.ndarray          # N x N           transition matrix
    log_a: np.ndarray      # N x N           np.log(a)                   (optimizer.py:328)
    emit: np.ndarray       # 625 x N         b[:, order[o]].sum(axis=1)  (optimizer.py:186)
    log_emit: np.ndarray   # 625 x N         np.log(emit[o])             (optimizer.py:329)
    pi_emit: np.ndarray    # 625 x N         pi * emit[o]                (optimizer.py:182)
    log_pi_emit: np.ndarray  # 625 x N       np.log(pi * emit[o])        (optimizer.py:182,323)


def _order():
    return [get_idx_state(i) for i in range(NOBS)]


_GROUPS = None


def _groups():
    """The 625 symbols grouped by expansion size k (1, 4, 16, 64, 256 N-free columns): per
    group the symbols and their [S, k] column-index table."""
    global _GROUPS
    if _GROUPS is None:
        by_k = {}
        for o, idx in enumerate(_order()):
            by_k.setdefault(len(idx), []).append((o, idx))
        _GROUPS = [(np.array([o for o, _ in v]), np.stack([idx for _, idx in v]))
                   for _, v in sorted(by_k.items())]
    return _GROUPS


def build_tables(a, b, pi) -> HmmTables:
    a = np.ascontiguousarray(a, dtype=np.float64)
    b = np.ascontiguousarray(b, dtype=np.float64)
    pi = np.ascontiguousarray(pi, dtype=np.float64)
    n = a.shape[0]
    if a.shape != (n, n) or b.shape != (n, 256) or pi.shape != (n,):
        raise ValueError(f"bad HMM shapes a{a.shape} b{b.shape} pi{pi.shape}")
    # emit[o] = b[:, order[o]].sum(axis=1) for every symbol, one fancy index + sum per
    # expansion size: each sum is the same contiguous pairwise reduction over the same k values
    # as the reference's per-symbol call, so the tables are bit-identical to it
    emit = np.empty((NOBS, n))
    for syms, idx in _groups():
        emit[syms] = b[:, idx].sum(axis=2).T
    with np.errstate(divide="ignore", invalid="ignore"):
        log_emit = np.log(emit)
        pi_emit = pi * emit
        log_pi_emit = np.log(pi_emit)
        log_a = np.log(a)
    return HmmTables(n, a, np.ascontiguousarray(log_a), emit, log_emit, pi_emit, log_pi_emit)
