"""Joint transition probabilities of two adjacent sites.

Restates get_joint_prob_mat.py:14-183 with run_markov_chain_AB.py:105-271 and
run_markov_chain_ABC.py:312-796.  A *path key* is a pair of site descriptors
((kind, i1, i2) left, (kind, i1, i2) right): which coalescence happened in which interval.
The chains keep one probability row vector (over CTMC states) per path key and advance all
of them interval by interval:

  * every key branches into the keys reachable in the interval (the 6 x 6 candidate table of
    run_markov_chain_ABC.py:354-405), skipping keys that already exist from an earlier
    interval;
  * a branch with at most one event per site is prob @ (diag(mask start) expm(Q dt)
    diag(mask end)) (run_markov_chain_ABC.py:9-14);
  * a branch with two coalescences at one site inside the interval needs the Van Loan
    integrals of every omega path between start and end (run_markov_chain_ABC.py:407-490);
  * after the last finite interval, keys still missing coalescences are closed with the
    deepest-interval integrals (run_markov_chain_ABC.py:512-796).

All matrix functions of one interval (and of the closing phase) are de-duplicated and handed
to the GPU backend as one batch; the per-key bookkeeping and the vector-matrix products stay
on the host, in the reference's order, so key insertion order and overwrite order match.
"""
from __future__ import annotations

from typing import Dict, List, Tuple

import numpy as np

from .paths import deepest_paths, vanloan_paths
from .statespace import (INVERTED_OMEGA_NONREV_COUNTS_3, masks_without, omega_nonrev_counts,
                         omega_of_key, state_space)

START = ((-1, -1, -1), (-1, -1, -1))  # get_joint_prob_mat.py:125


def _interval_lengths(cut) -> List[float]:
    """cut[i+1] - cut[i] (cutpoints.py:48-65 get_times)."""
    return [cut[i + 1] - cut[i] for i in range(len(cut) - 1)]


def combine_states(sd1, sd2, sd_sum, p1: np.ndarray, p2: np.ndarray) -> np.ndarray:
    """Initial vector of the merged chain: product measure of two independent chains, each
    merged state relabelled by first appearance (combine_states.py:5-90)."""
    out = np.zeros(sd_sum.n, dtype=np.float64)
    for s1, i1 in sd1.index.items():
        h1 = len(s1) // 2
        for s2, i2 in sd2.index.items():
            h2 = len(s2) // 2
            seen1, seen2, lab, nxt = {}, {}, [], 1
            for part, seen in ((s1[:h1], seen1), (s2[:h2], seen2), (s1[h1:], seen1),
                               (s2[h2:], seen2)):
                for v in part:
                    if v not in seen:
                        seen[v] = nxt
                        nxt += 1
                    lab.append(seen[v])
            out[sd_sum.index[tuple(lab)]] = p1[0, i1] * p2[0, i2]
    return out.reshape(1, -1)


def _branch_rows_ab(side, step):
    """Candidate descriptors of one site in the AB epoch (run_markov_chain_AB.py:131-140)."""
    return [side, (0, step, side[2]) if side[0] == -1 else side]


def _branch_rows_abc(side, step):
    """Candidate descriptors of one site in an ABC interval (run_markov_chain_ABC.py:354-390)."""
    k, i1, i2 = side
    fresh = k == -1
    return [
        side,
        (k, step, step) if fresh else side,
        (1, step, i2) if fresh else side,
        (2, step, i2) if fresh else side,
        (3, step, i2) if fresh else side,
        (k, i1, step) if (k != -1 and i2 == -1) else side,
    ]


def run_chain_ab(Q, times, masks, probs: Dict, n_int, la) -> Dict:
    """run_markov_chain_AB.py:105-271: two-species chain over the n_int AB intervals."""
    for step in range(n_int):
        E = la.expm([Q * times[step]])[0]
        og = list(probs.keys())
        ogs = set(og)
        updates = []
        for path in og:
            pm = probs[path]
            lrows = _branch_rows_ab(path[0], step)
            rrows = _branch_rows_ab(path[1], step)
            for l in lrows:
                for r in rrows:
                    key = (tuple(int(x) for x in l), tuple(int(x) for x in r))
                    if key in ogs and key != path:
                        continue
                    me = masks[omega_of_key(key)].astype(np.float64)
                    if step == 0:
                        res = (pm @ E) * me  # run_markov_chain_AB.py:9-12
                    else:
                        ms = masks[omega_of_key(path)].astype(np.float64)
                        res = (pm * ms) @ E * me
                    updates.append((key, res))
            if step > 0:  # steps >= 1 write per path (run_markov_chain_AB.py:262-270)
                for key, res in updates:
                    probs[key] = res
                updates = []
        for key, res in updates:  # step 0 writes after the loop (only START exists)
            probs[key] = res
    return probs


def run_chain_abc(Q, times, ss, probs: Dict, n_int, la) -> Dict:
    """run_markov_chain_ABC.py:312-796: three-species chain, n_int - 1 finite intervals and
    the closing deepest interval; returns {hidden-state pair: probability}."""
    masks = ss.omega_masks
    nrc = omega_nonrev_counts(3)
    inv = INVERTED_OMEGA_NONREV_COUNTS_3
    for step in range(n_int - 1):
        dt = times[step]
        E = la.expm([Q * dt])[0]
        og = list(probs.keys())
        ogs = set(og)
        plan = []  # per path: [(key, ms, me, kind, payload)]
        vl_needed = {}
        for path in og:
            lrows = _branch_rows_abc(path[0], step)
            rrows = _branch_rows_abc(path[1], step)
            plain, vl = [], []
            om_s = omega_of_key(path)
            for l in lrows:
                lt = tuple(int(x) for x in l)
                for r in rrows:
                    rt = tuple(int(x) for x in r)
                    key = (lt, rt)
                    if key in ogs and key != path:
                        continue
                    om_e = omega_of_key(key)
                    double_l = lt[0] != 0 and lt[1] == lt[2] and lt[1] != -1
                    double_r = rt[0] != 0 and rt[1] == rt[2] and rt[1] != -1
                    if double_l or double_r:
                        groups = vanloan_paths(om_s, om_e, nrc, inv, lt, rt, lt, rt)
                        for key6, sub in groups:
                            for p in sub:
                                vl_needed[p] = None
                            vl.append((key6, sub, om_s, om_e))
                    else:
                        plain.append((key, om_s, om_e))
            plan.append((path, plain, vl))
        # one batch of Van Loan exponentials for the whole interval
        vl_list = list(vl_needed.keys())
        for p, S in zip(vl_list, la.vanloan(Q, dt, masks, vl_list)):
            vl_needed[p] = S
        for path, plain, vl in plan:
            pm = probs[path]
            writes = []
            for key, om_s, om_e in plain:
                ms = masks[om_s].astype(np.float64)
                me = masks[om_e].astype(np.float64)
                writes.append((key, (pm * ms) @ E * me))
            for key6, sub, om_s, om_e in vl:
                S = vl_needed[sub[0]].copy()
                for p in sub[1:]:
                    S = S + vl_needed[p]
                ms = masks[om_s].astype(np.float64)
                me = masks[om_e].astype(np.float64)
                writes.append(((key6[:3], key6[3:]), (pm * ms) @ S * me))
            for key, v in writes:  # plain results first, then Van Loan ones
                probs[key] = v
    return _close_deepest(Q, ss, probs, n_int, la)


def _close_deepest(Q, ss, probs: Dict, n_int, la) -> Dict:
    """The unbounded last interval (run_markov_chain_ABC.py:512-796)."""
    masks = ss.omega_masks
    nrc = omega_nonrev_counts(3)
    inv = INVERTED_OMEGA_NONREV_COUNTS_3
    absorbing = (7, 7)
    keep = ~masks[absorbing]
    Qn = Q[keep][:, keep]
    masks_n = masks_without(masks, absorbing)
    last = n_int - 1
    out: Dict = {}
    tasks = []  # (insertion position, key6, [paths], acc_prob)
    order: List = []  # sequence of ("sum", key, value) / ("deep", task index)
    for path in list(probs.keys()):
        l, r = path
        pm = probs[path]
        l_done, r_done = all(x != -1 for x in l), all(x != -1 for x in r)
        l_half = l[2] == -1 and all(x != -1 for x in l[:2])
        r_half = r[2] == -1 and all(x != -1 for x in r[:2])
        l_none, r_none = all(x == -1 for x in l), all(x == -1 for x in r)
        if l_done and r_done:
            order.append(("sum", path, pm))
            continue
        if l_done and r_half:
            order.append(("sum", (l, (r[0], r[1], last)), pm))
            continue
        if l_half and r_done:
            order.append(("sum", ((l[0], l[1], last), r), pm))
            continue
        if l_half and r_half:
            order.append(("sum", ((l[0], l[1], last), (r[0], r[1], last)), pm))
            continue
        if l_done and r_none:
            new = (l, (r[0], last, last))
        elif l_half and r_none:
            new = ((l[0], l[1], last), (r[0], last, last))
        elif l_none and r_done:
            new = ((l[0], last, last), r)
        elif l_none and r_half:
            new = ((l[0], last, last), (r[0], r[1], last))
        elif l_none and r_none:
            new = ((l[0], last, last), (r[0], last, last))
        else:
            continue  # the reference drops keys of any other shape
        groups = deepest_paths(omega_of_key(path), absorbing, nrc, inv, new)
        for key6, sub in groups:
            if all(x == 0 for x in key6):  # run_markov_chain_ABC.py:150 stops at a zero key
                break
            tasks.append((key6, sub, pm[:, keep]))
            order.append(("deep", len(tasks) - 1))
    needed = {}
    for _, sub, _ in tasks:
        for p in sub:
            needed[p] = None
    plist = list(needed.keys())
    for p, D in zip(plist, la.deepest(Qn, masks_n, plist)):
        needed[p] = D
    for item in order:
        if item[0] == "sum":
            out[tuple(tuple(int(v) for v in s) for s in item[1])] = np.sum(item[2])
        else:
            key6, sub, acc = tasks[item[1]]
            D = needed[sub[0]].copy()
            for p in sub[1:]:
                D = D + needed[p]
            out[(tuple(key6[:3]), tuple(key6[3:]))] = np.sum(acc @ D)
    return out


def joint_prob_mat(t_A, t_B, t_AB, t_C, rho_A, rho_B, rho_AB, rho_C, rho_ABC, coal_A, coal_B,
                   coal_AB, coal_C, coal_ABC, n_int_AB, n_int_ABC, cut_AB, cut_ABC,
                   la=None) -> Dict:
    """get_joint_prob_mat (get_joint_prob_mat.py:14-183): {(state_left, state_right): p}."""
    if la is None:
        from .linalg import DeviceLinalg
        la = DeviceLinalg()
    s1, s2, s3 = state_space(1), state_space(2), state_space(3)
    Qa = s1.rate_matrix(coal_A, rho_A)
    Qb = s1.rate_matrix(coal_B, rho_B)
    Qc = s1.rate_matrix(coal_C, rho_C)
    Qab = s2.rate_matrix(coal_AB, rho_AB)
    Qabc = s3.rate_matrix(coal_ABC, rho_ABC)
    pi1 = np.zeros(2)
    pi1[s1.index[(1, 1)]] = 1.0
    Ea, Eb, Ec = la.expm([Qa * t_A, Qb * t_B, Qc * t_C])
    fa = (pi1 @ Ea).reshape(1, -1)
    fb = (pi1 @ Eb).reshape(1, -1)
    fc = (pi1 @ Ec).reshape(1, -1)
    pi_ab = {START: combine_states(s1, s1, s2, fa, fb)}
    ab = run_chain_ab(Qab, _interval_lengths(cut_AB), s2.omega_masks, pi_ab, n_int_AB, la)
    pi_abc = {path: combine_states(s2, s1, s3, p, fc) for path, p in ab.items()}
    return run_chain_abc(Qabc, _interval_lengths(cut_ABC), s3, pi_abc, n_int_ABC, la)
