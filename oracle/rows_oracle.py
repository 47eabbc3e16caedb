"""NumPy restatement of the reference's standalone sweep matrices — TEST INFRASTRUCTURE ONLY
(see oracle/__init__.py): the checker of itr_block_rows / itr_backtrack_rows
(itrails_amd/csrc/rows.hip), never a product path.

Each function restates one reference function expression by expression on the per-symbol
tables of itrails_amd/tables.py (`emit[o]` = b[:, order[o]].sum(axis=1), `log_pi_emit[o]` =
np.log(pi * emit[o]), `log_a` = np.log(a), `log_emit[o]` = np.log(emit[o])).  Pure-Python
loops over columns: small blocks only.  Pinned by tests/test_oracle.py against the
reference-generated goldens (tests/golden/sweep_*.npz: log-likelihoods, paths, posteriors).
"""
from __future__ import annotations

import numpy as np


def forward(t, V) -> np.ndarray:
    """optimizer.py:165-188."""
    alpha = np.zeros((V.shape[0], t.n))
    alpha[0, :] = t.log_pi_emit[V[0]]
    for k in range(1, V.shape[0]):
        x = alpha[k - 1, :].max()
        alpha[k, :] = np.log((np.exp(alpha[k - 1] - x) @ t.a) * t.emit[V[k]]) + x
    return alpha


def loglik_from_alpha(alpha) -> float:
    """optimizer.py:160-162."""
    x = alpha[-1, :].max()
    return float(np.log(np.exp(alpha[len(alpha) - 1] - x).sum()) + x)


def backward(t, V) -> np.ndarray:
    """optimizer.py:191-213 (the reference's (beta * e) @ a)."""
    beta = np.zeros((V.shape[0], t.n))
    for k in range(V.shape[0] - 2, -1, -1):
        x = beta[k + 1, :].max()
        beta[k, :] = np.log((np.exp(beta[k + 1] - x) * t.emit[V[k + 1]]) @ t.a) + x
    return beta


def post_from_rows(alpha, beta) -> np.ndarray:
    """optimizer.py:231-238."""
    p = alpha + beta
    m = p.max(1).reshape(-1, 1)
    return np.exp(p - m) / np.exp(p - m).sum(1).reshape(-1, 1)


def viterbi(t, V):
    """optimizer.py:305-333: (omega, prev)."""
    T = V.shape[0]
    omega = np.zeros((T, t.n))
    omega[0, :] = t.log_pi_emit[V[0]]
    prev = np.zeros((T - 1, t.n))
    with np.errstate(invalid="ignore"):
        for k in range(1, T):
            pm = omega[k - 1][:, np.newaxis] + t.log_a + t.log_emit[V[k]]
            prev[k - 1, :] = np.argmax(pm, axis=0)
            omega[k, :] = np.max(pm, axis=0)
    return omega, prev


def backtrack_viterbi(omega, prev) -> np.ndarray:
    """optimizer.py:336-354."""
    T = omega.shape[0]
    S = np.zeros(T)
    last = np.argmax(omega[T - 1, :])
    S[0] = last
    for j, i in enumerate(range(T - 2, -1, -1)):
        S[j + 1] = prev[i, int(last)]
        last = prev[i, int(last)]
    return np.flip(S)
