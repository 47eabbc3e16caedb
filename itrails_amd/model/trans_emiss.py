"""trans_emiss_calc (get_trans_emiss.py:8-170): the HMM (a, b, pi) of the iTRAILS model.

Parameters are scaled to coalescent units of N_ref = N_ABC exactly as
get_trans_emiss.py:62-89; cutpoints default to the exponential quantiles
(cutpoints.py:5-45); the joint two-site probabilities J come from the CTMC chains
(chains.py) and the emission rows from emissions.py.  Hidden states are sorted by their
(topology, i, j) tuple (get_trans_emiss.py:150-153); pi = J.sum(1) and a = J / pi
(get_trans_emiss.py:166-168).
"""
from __future__ import annotations

import numpy as np

from .chains import joint_prob_mat, prefetch_vanloan
from .statespace import state_space
from .emissions import cutpoints_AB, cutpoints_ABC, emission_rows, state_specs

_NT = ["A", "C", "T", "G"]
OBSERVED_NAMES = {i: _NT[i >> 6] + _NT[(i >> 4) & 3] + _NT[(i >> 2) & 3] + _NT[i & 3]
                  for i in range(256)}


_PAIR_INDEX: dict = {}


def _pair_index(n_int_AB, n_int_ABC, hidden, J):
    """Row / column of every joint-probability key (in J's order) in the sorted hidden-state
    order.  J's keys come in the same order at every rebuild of one model size (the chain's
    planned enumeration), so the index arrays are built once per size and reused while the
    states and the keys' count and ends match."""
    keys = list(J.keys())
    k = (n_int_AB, n_int_ABC)
    c = _PAIR_INDEX.get(k)
    if c is None or c[0] != hidden or c[1] != keys:
        index = {s: i for i, s in enumerate(hidden)}
        r = np.fromiter((index[tuple(a)] for a, _ in keys), dtype=np.int64, count=len(keys))
        q = np.fromiter((index[tuple(d)] for _, d in keys), dtype=np.int64, count=len(keys))
        c = _PAIR_INDEX[k] = (list(hidden), keys, r, q)
    return c[2], c[3]


def trans_emiss_calc(t_A, t_B, t_C, t_2, t_upper, t_out, N_AB, N_ABC, r, n_int_AB,
                     n_int_ABC, cut_AB="standard", cut_ABC="standard", la=None):
    """-> (a, b, pi, hidden_names, observed_names), the reference's return tuple."""
    if la is None:
        from .linalg import DeviceLinalg
        la = DeviceLinalg()
    N_ref = N_ABC
    t_A = t_A / N_ref
    t_B = t_B / N_ref
    t_AB = t_2 / N_ref
    t_C = t_C / N_ref
    t_upper = t_upper / N_ref
    t_out = t_out / N_ref
    rho = N_ref * r
    coal_AB = N_ref / N_AB
    coal_ABC = N_ref / N_ABC
    mu = N_ref * (4 / 3)
    if isinstance(cut_AB, str):
        if cut_AB != "standard":
            raise ValueError(f"unknown cutpoint scheme {cut_AB!r}")
        cut_AB = cutpoints_AB(n_int_AB, t_AB, coal_AB)
    if isinstance(cut_ABC, str):
        if cut_ABC != "standard":
            raise ValueError(f"unknown cutpoint scheme {cut_ABC!r}")
        cut_ABC = cutpoints_ABC(n_int_ABC, coal_ABC)

    # the three-species chain's Van Loan work (the bulk of the build's device time) starts
    # first, on a side stream, and runs while the host builds the emission tables and the
    # two-species chain
    prefetch_vanloan(state_space(3).rate_matrix(coal_ABC, rho),
                     [cut_ABC[i + 1] - cut_ABC[i] for i in range(len(cut_ABC) - 1)],
                     state_space(3), n_int_ABC, la)
    specs = state_specs(t_A, t_B, t_AB, t_C, t_upper, t_out, coal_AB, coal_ABC, n_int_AB,
                        n_int_ABC, mu, mu, mu, mu, mu, mu, cut_AB, cut_ABC)
    states, rows = emission_rows(specs, la=la)
    J = joint_prob_mat(t_A, t_B, t_AB, t_C, rho, rho, rho, rho, rho, coal_AB, coal_AB,
                       coal_AB, coal_AB, coal_ABC, n_int_AB, n_int_ABC, cut_AB, cut_ABC, la=la)
    order = sorted(range(len(states)), key=lambda i: states[i])
    hidden = [states[i] for i in order]
    b = rows[order]
    n = len(hidden)
    rows_idx, cols_idx = _pair_index(n_int_AB, n_int_ABC, hidden, J)
    T = np.zeros((n, n))
    T[rows_idx, cols_idx] = np.fromiter(J.values(), dtype=np.float64, count=len(J))
    pi = T.sum(axis=1)
    a = T / pi[:, None]
    return a, b, pi, dict(enumerate(hidden)), dict(OBSERVED_NAMES)
