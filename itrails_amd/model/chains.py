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

from functools import lru_cache
from typing import Dict, List, Tuple

import numpy as np

from .paths import deepest_paths, vanloan_paths
from .statespace import (INVERTED_OMEGA_NONREV_COUNTS_3, masks_without, omega_nonrev_counts,
                         omega_of_key, state_space)

START = ((-1, -1, -1), (-1, -1, -1))  # get_joint_prob_mat.py:125


def _interval_lengths(cut) -> List[float]:
    """cut[i+1] - cut[i] (cutpoints.py:48-65 get_times)."""
    return [cut[i + 1] - cut[i] for i in range(len(cut) - 1)]


_COMBINE: Dict = {}


def combine_states(sd1, sd2, sd_sum, p1: np.ndarray, p2: np.ndarray) -> np.ndarray:
    """Initial vector of the merged chain: product measure of two independent chains, each
    merged state relabelled by first appearance (combine_states.py:5-90).  The relabelling
    depends only on the three state spaces and is computed once."""
    key = (id(sd1), id(sd2), id(sd_sum))
    m = _COMBINE.get(key)
    if m is None:
        i1s, i2s, tgt = [], [], []
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
                i1s.append(i1)
                i2s.append(i2)
                tgt.append(sd_sum.index[tuple(lab)])
        m = (np.asarray(i1s), np.asarray(i2s), np.asarray(tgt))
        if len(set(tgt)) != len(tgt):
            raise AssertionError("combine_states: relabelling is not one-to-one")
        _COMBINE[key] = m
    i1, i2, tgt = m
    out = np.zeros(sd_sum.n, dtype=np.float64)
    out[tgt] = p1[0, i1] * p2[0, i2]
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
    """run_markov_chain_AB.py:105-271: two-species chain over the n_int AB intervals (every
    interval's propagator expm(Q dt) requested as one batch up front).

    Within a step every product reads a step-start row: a path writes only new keys or its
    own (keys of the step's other paths are skipped), and after its reads.  So a step is one
    batched product over its (path, key) updates, applied in the reference's write order —
    planned once per (n_int, starting keys) from the key structure alone (_plan_ab)."""
    Es = la.expm([Q * times[step] for step in range(n_int)])
    keys0 = list(probs.keys())
    pk = (n_int, tuple(keys0), id(masks))
    plan = _AB_PLANS.get(pk)
    if plan is None:
        plan = _AB_PLANS[pk] = _plan_ab(masks, keys0, n_int)
    V = np.concatenate([np.asarray(probs[k], dtype=np.float64).reshape(1, -1) for k in keys0])
    for step, (pidx, ms, me, take_old, take_upd) in enumerate(plan.steps):
        A = V[pidx]
        if step > 0:
            A = A * ms  # (pm * ms) @ E * me, run_markov_chain_AB.py:262-270
        R = (A @ Es[step]) * me  # step 0: (pm @ E) * me, run_markov_chain_AB.py:9-12
        Vn = np.empty((len(take_old), V.shape[1]))
        old = take_old >= 0
        Vn[old] = V[take_old[old]]
        Vn[~old] = R[take_upd[~old]]
        V = Vn
    return {k: V[i:i + 1] for i, k in enumerate(plan.keys)}


_AB_PLANS: Dict = {}


class _ABPlan:
    __slots__ = ("steps", "keys")


def _plan_ab(masks, keys0, n_int) -> _ABPlan:
    """The two-species chain's structure: per step the updates (source row, start mask,
    end mask) of every (path, candidate key) the reference evaluates, and the resulting key
    order with each key's source (a kept row or an update; later writes win, a key keeps
    its first-insertion position like the reference's dict)."""
    plan = _ABPlan()
    plan.steps = []
    keys = list(keys0)
    for step in range(n_int):
        ogs = set(keys)
        pidx, ms, me, ukeys = [], [], [], []
        for i, path in enumerate(keys):
            for l in _branch_rows_ab(path[0], step):
                for r in _branch_rows_ab(path[1], step):
                    key = (tuple(int(x) for x in l), tuple(int(x) for x in r))
                    if key in ogs and key != path:
                        continue
                    pidx.append(i)
                    ms.append(masks[omega_of_key(path)])
                    me.append(masks[omega_of_key(key)])
                    ukeys.append(key)
        src = {k: (i, -1) for i, k in enumerate(keys)}
        for u, k in enumerate(ukeys):
            src[k] = (-1, u)
        order = list(src.keys())
        plan.steps.append((np.asarray(pidx, dtype=np.int64),
                           np.asarray(ms, dtype=np.float64).reshape(len(pidx), -1),
                           np.asarray(me, dtype=np.float64).reshape(len(pidx), -1),
                           np.asarray([src[k][0] for k in order], dtype=np.int64),
                           np.asarray([src[k][1] for k in order], dtype=np.int64)))
        keys = order
    plan.keys = keys
    return plan


_LAST_PLAN: Dict = {}  # n_int -> the plan of the last build (its keys recur every rebuild)


def prefetch_vanloan(Q, times, ss, n_int, la) -> None:
    """Start the three-species chain's Van Loan evaluation (all intervals, their propagators)
    on a side stream before the host-heavy parts of the build (emissions, the AB chain) run,
    when the previous build of this size left its plan (every optimizer rebuild after the
    first).  _run_chain_abc_device picks the result up if the plan and inputs match."""
    import torch
    plan = _LAST_PLAN.get(n_int)
    la._prefetch = None
    if plan is None or not hasattr(la, "vanloan_batch") or getattr(la, "world", 1) > 1 \
            or not getattr(la.dev, "type", "") == "cuda":
        return
    tab = _device_tables(plan, Q, ss, la)
    I = len(plan.intervals)
    t = np.asarray([times[i] for i in range(I)] * 2, dtype=np.float64)
    side = getattr(la, "_side", None)
    if side is None:
        side = la._side = torch.cuda.Stream(device=la.dev)
    side.wait_stream(torch.cuda.current_stream(la.dev))
    with torch.cuda.stream(side):
        S = la.vanloan_batch(Q, tab["mask_u8"], t, tab["job"], tab["off"], tab["pm"])
        ev = torch.cuda.Event()
        ev.record(side)
    la._prefetch = (plan, np.array(Q, copy=True), t, S, ev)


def _take_prefetch(plan, Q, t, la):
    """The prefetched Van Loan results if they were computed for exactly these inputs."""
    import torch
    pre = getattr(la, "_prefetch", None)
    la._prefetch = None
    if pre is None:
        return None
    p, Qp, tp, S, ev = pre
    if p is not plan or not np.array_equal(Qp, Q) or not np.array_equal(tp, t):
        return None
    cur = torch.cuda.current_stream(la.dev)
    cur.wait_event(ev)
    S.record_stream(cur)
    return S


def run_chain_abc(Q, times, ss, probs: Dict, n_int, la) -> Dict:
    """run_markov_chain_ABC.py:312-796: three-species chain, n_int - 1 finite intervals and
    the closing deepest interval; returns {hidden-state pair: probability}.

    The branching structure (which keys exist, which branch reaches which key through which
    omega classes and Van Loan paths) depends only on n_int and the incoming keys, so it is
    planned once (`_abc_plan`, cached: every objective evaluation of the optimizer reuses
    it) and each build only runs the numbers: per interval one expm, one Van Loan batch,
    one stacked GEMM for the plain branches and one per Van Loan path group."""
    plan = _abc_plan(n_int, tuple(probs.keys()))
    if plan is None:  # an interval whose path-by-path order matters: the dict form
        return _run_chain_abc_dicts(Q, times, ss, probs, n_int, la)
    _LAST_PLAN[n_int] = plan
    if hasattr(la, "vanloan_batch"):
        return _run_chain_abc_device(plan, Q, times, ss, probs, la)
    return _run_chain_abc_planned(plan, Q, times, ss, probs, la)


def _run_chain_abc_dicts(Q, times, ss, probs: Dict, n_int, la) -> Dict:
    """run_chain_abc on dictionaries, interval by interval (the reference's form)."""
    masks = ss.omega_masks
    fmask = {k: m.astype(np.float64) for k, m in masks.items()}
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
        # every product of the interval as stacked row blocks: (pm * ms) @ E * me for the
        # plain branches (one GEMM), (pm * ms) @ sum(S over the group's omega paths) * me
        # for the Van Loan groups (one GEMM per distinct path group)
        plain_rows, plain_out = [], []
        vl_rows: Dict[tuple, list] = {}
        for pi_, (path, plain, vl) in enumerate(plan):
            pm = probs[path][0]
            for k, (key, om_s, om_e) in enumerate(plain):
                plain_out.append((pi_, k, om_e))
                plain_rows.append(pm * fmask[om_s])
            for k, (key6, sub, om_s, om_e) in enumerate(vl):
                vl_rows.setdefault(tuple(sub), []).append((pi_, k, om_s, om_e))
        # The reference updates path by path, so a later path reads an earlier path's write
        # if that write lands on its key; the stacked products read every path first, which
        # is the same only without such a hazard (otherwise: the path-by-path order).
        pos = {path: i for i, (path, _, _) in enumerate(plan)}
        hazard = any(pos.get(key, -1) > i for i, (path, plain, vl) in enumerate(plan)
                     for key in [k for k, _, _ in plain] + [(k6[:3], k6[3:]) for k6, _, _, _ in vl])
        if hazard:
            _products_in_order(plan, probs, E, vl_needed, fmask)
            continue
        res_plain = {}
        if plain_rows:
            R = la.rowmat(np.stack(plain_rows), E)
            for (pi_, k, om_e), row in zip(plain_out, R):
                res_plain[(pi_, k)] = (row * fmask[om_e]).reshape(1, -1)
        res_vl = {}
        for sub, items in vl_rows.items():
            S = vl_needed[sub[0]].copy()
            for p in sub[1:]:
                S = S + vl_needed[p]
            V = np.stack([probs[plan[pi_][0]][0] * fmask[om_s] for pi_, _, om_s, _ in items])
            R = V @ S
            for (pi_, k, _, om_e), row in zip(items, R):
                res_vl[(pi_, k)] = (row * fmask[om_e]).reshape(1, -1)
        for pi_, (path, plain, vl) in enumerate(plan):
            for k, (key, _, _) in enumerate(plain):  # plain results first, then Van Loan ones
                probs[key] = res_plain[(pi_, k)]
            for k, (key6, _, _, _) in enumerate(vl):
                probs[(key6[:3], key6[3:])] = res_vl[(pi_, k)]
    return _close_deepest(Q, ss, probs, n_int, la)


class _IntervalPlan:
    __slots__ = ("vl_paths", "plain", "groups")

    def __init__(self, vl_paths, plain, groups):
        self.vl_paths = vl_paths   # distinct Van Loan omega paths of the interval
        self.plain = plain         # (src rows, start omega ids, end omega ids, dst rows)
        self.groups = groups       # [(path ids, src, start ids, end ids, dst)] per path group


class _ABCPlan:
    __slots__ = ("nrows", "omegas", "intervals", "close_paths", "close_order", "close_groups",
                 "close_sum_rows", "dev")


@lru_cache(maxsize=16)
def _abc_plan(n_int: int, keys0: tuple):
    """The structural plan of run_chain_abc for n_int intervals and the incoming keys (in
    their order): per interval the branch table as row-index arrays, then the closing phase.
    None if some interval has a path-by-path ordering hazard (a later path reading a key an
    earlier path of the same interval wrote)."""
    nrc = omega_nonrev_counts(3)
    inv = INVERTED_OMEGA_NONREV_COUNTS_3
    rows = {k: i for i, k in enumerate(keys0)}
    keys = list(keys0)
    om_ids: Dict = {}

    def oid(om):
        if om not in om_ids:
            om_ids[om] = len(om_ids)
        return om_ids[om]

    def row_of(key):
        if key not in rows:
            rows[key] = len(keys)
            keys.append(key)
        return rows[key]

    intervals = []
    for step in range(n_int - 1):
        og = list(keys)
        ogs = set(og)
        pos = {k: i for i, k in enumerate(og)}
        writes = []  # (dst key, kind, payload) in the reference's write order
        vl_index: Dict = {}
        for pi_, path in enumerate(og):
            om_s = omega_of_key(path)
            plain, vl = [], []
            for l in _branch_rows_abc(path[0], step):
                lt = tuple(int(x) for x in l)
                for r in _branch_rows_abc(path[1], step):
                    rt = tuple(int(x) for x in r)
                    key = (lt, rt)
                    if key in ogs and key != path:
                        continue
                    om_e = omega_of_key(key)
                    double_l = lt[0] != 0 and lt[1] == lt[2] and lt[1] != -1
                    double_r = rt[0] != 0 and rt[1] == rt[2] and rt[1] != -1
                    if double_l or double_r:
                        for key6, sub in vanloan_paths(om_s, om_e, nrc, inv, lt, rt, lt, rt):
                            for p in sub:
                                vl_index.setdefault(p, len(vl_index))
                            vl.append(((key6[:3], key6[3:]), ("vl", tuple(sub), om_s, om_e)))
                    else:
                        plain.append((key, ("plain", None, om_s, om_e)))
            for key, how in plain + vl:
                if pos.get(key, -1) > pi_:
                    return None
                writes.append((key, path, how))
        last = {}
        for w, (key, _, _) in enumerate(writes):  # a later write of the same key wins
            last[key] = w
        src_rows = [rows[path] for _, path, _ in writes]
        dst_rows = [row_of(key) for key, _, _ in writes]
        pl = [[], [], [], []]
        gr: Dict = {}
        for w, (key, path, (kind, sub, om_s, om_e)) in enumerate(writes):
            if last[key] != w:
                continue
            if kind == "plain":
                tgt = pl
            else:
                tgt = gr.setdefault(sub, [[], [], [], []])
            tgt[0].append(src_rows[w])
            tgt[1].append(oid(om_s))
            tgt[2].append(oid(om_e))
            tgt[3].append(dst_rows[w])
        arr = lambda v: np.asarray(v, dtype=np.int64)  # noqa: E731
        groups = [(arr([vl_index[p] for p in sub]), arr(g[0]), arr(g[1]), arr(g[2]), arr(g[3]))
                  for sub, g in gr.items()]
        intervals.append(_IntervalPlan(list(vl_index), tuple(arr(v) for v in pl), groups))

    # the closing (unbounded) interval: run_markov_chain_ABC.py:512-796
    absorbing = (7, 7)
    last_i = n_int - 1
    close_order = []       # (out key, "sum", sum index) / (out key, "deep", task index)
    sum_rows = []
    task_rows, task_subs = [], []
    dp_index: Dict = {}
    for path in keys:
        l, r = path
        row = rows[path]
        l_done, r_done = all(x != -1 for x in l), all(x != -1 for x in r)
        l_half = l[2] == -1 and all(x != -1 for x in l[:2])
        r_half = r[2] == -1 and all(x != -1 for x in r[:2])
        l_none, r_none = all(x == -1 for x in l), all(x == -1 for x in r)
        summed = None
        if l_done and r_done:
            summed = path
        elif l_done and r_half:
            summed = (l, (r[0], r[1], last_i))
        elif l_half and r_done:
            summed = ((l[0], l[1], last_i), r)
        elif l_half and r_half:
            summed = ((l[0], l[1], last_i), (r[0], r[1], last_i))
        if summed is not None:
            close_order.append((tuple(tuple(int(v) for v in sd) for sd in summed), "sum",
                                len(sum_rows)))
            sum_rows.append(row)
            continue
        if l_done and r_none:
            new = (l, (r[0], last_i, last_i))
        elif l_half and r_none:
            new = ((l[0], l[1], last_i), (r[0], last_i, last_i))
        elif l_none and r_done:
            new = ((l[0], last_i, last_i), r)
        elif l_none and r_half:
            new = ((l[0], last_i, last_i), (r[0], r[1], last_i))
        elif l_none and r_none:
            new = ((l[0], last_i, last_i), (r[0], last_i, last_i))
        else:
            continue  # the reference drops keys of any other shape
        for key6, sub in deepest_paths(omega_of_key(path), absorbing, nrc, inv, new):
            if all(x == 0 for x in key6):  # run_markov_chain_ABC.py:150 stops at a zero key
                break
            for p in sub:
                dp_index.setdefault(p, len(dp_index))
            close_order.append(((tuple(key6[:3]), tuple(key6[3:])), "deep", len(task_rows)))
            task_rows.append(row)
            task_subs.append(tuple(sub))
    cg: Dict = {}
    for t, sub in enumerate(task_subs):
        cg.setdefault(sub, []).append(t)
    plan = _ABCPlan()
    plan.nrows = len(keys)
    plan.omegas = [om for om, _ in sorted(om_ids.items(), key=lambda kv: kv[1])]
    plan.intervals = intervals
    plan.close_paths = list(dp_index)
    plan.close_order = close_order
    plan.close_sum_rows = np.asarray(sum_rows, dtype=np.int64)
    plan.close_groups = [(np.asarray([dp_index[p] for p in sub], dtype=np.int64),
                          np.asarray(ts, dtype=np.int64),
                          np.asarray([task_rows[t] for t in ts], dtype=np.int64))
                         for sub, ts in cg.items()]
    plan.dev = {}
    return plan


def _run_chain_abc_planned(plan, Q, times, ss, probs: Dict, la) -> Dict:
    """The numbers of run_chain_abc on a structural plan: key rows of one matrix."""
    masks = ss.omega_masks
    n = Q.shape[0]
    P = np.zeros((plan.nrows, n))
    for i, v in enumerate(probs.values()):
        P[i] = v[0]
    F = np.stack([masks[om].astype(np.float64) for om in plan.omegas]) if plan.omegas else \
        np.zeros((0, n))
    for step, ip in enumerate(plan.intervals):
        dt = times[step]
        E = la.expm([Q * dt])[0]
        S = la.vanloan(Q, dt, masks, ip.vl_paths) if ip.vl_paths else []
        results = []
        src, oms, ome, dst = ip.plain
        if src.size:
            results.append((dst, la.rowmat(P[src] * F[oms], E) * F[ome]))
        for pids, src, oms, ome, dst in ip.groups:
            M = S[pids[0]].copy()
            for j in pids[1:]:
                M = M + S[j]
            results.append((dst, (P[src] * F[oms]) @ M * F[ome]))
        for dst, R in results:  # every read above happened before these writes
            P[dst] = R
    absorbing = (7, 7)
    keep = ~masks[absorbing]
    Qn = Q[keep][:, keep]
    masks_n = masks_without(masks, absorbing)
    D = la.deepest(Qn, masks_n, plan.close_paths) if plan.close_paths else []
    sums = P[plan.close_sum_rows].sum(axis=1) if plan.close_sum_rows.size else np.zeros(0)
    deep = np.zeros(sum(len(t) for _, t, _ in plan.close_groups))
    for pids, tasks, rws in plan.close_groups:
        M = D[pids[0]].copy()
        for j in pids[1:]:
            M = M + D[j]
        deep[tasks] = (P[rws][:, keep] @ M).sum(axis=1)
    out: Dict = {}
    for key, kind, k in plan.close_order:
        out[key] = float(sums[k]) if kind == "sum" else float(deep[k])
    return out


class _DevInterval:
    __slots__ = ("e_idx", "vl0", "vl1", "plain", "ng", "sum_steps", "rows", "rmax")


class _GroupSums:
    """The path groups of a set of group matrices M[g] = S[p_g0] + S[p_g1] + ...: as CSR
    (int32 offsets + path indices, one itr_group_sum launch on the device) and as the
    sequential steps of the same sums (step k adds the k-th path of every group that has
    one) for a CPU-tensor rehearsal of the routing (tests)."""
    __slots__ = ("ng", "off", "paths", "steps")


def _group_tables(dev, pids_list, rows_of_group):
    """Index tensors of a set of path groups: the path sums of each group's matrix (the
    reference's left-to-right S = S_0 + S_1 + ..., run_markov_chain_ABC.py:478-486) and, for
    the row products, every row's (group, slot) in a zero-padded [groups, rmax] layout."""
    import torch
    gsum = _GroupSums()
    gsum.ng = len(pids_list)
    lens = [len(p) for p in pids_list]
    gsum.off = torch.as_tensor(np.concatenate([[0], np.cumsum(lens)]).astype(np.int32),
                               device=dev)
    flat = [int(x) for p in pids_list for x in p]
    gsum.paths = torch.as_tensor(np.asarray(flat, dtype=np.int32), device=dev)
    gsum.steps = []
    if torch.device(dev).type == "cpu":
        kmax = max(lens, default=0)
        for k in range(kmax):
            gs = [g for g, p in enumerate(pids_list) if len(p) > k]
            ps = [int(pids_list[g][k]) for g in gs]
            gsum.steps.append((torch.as_tensor(gs, dtype=torch.long, device=dev),
                               torch.as_tensor(ps, dtype=torch.long, device=dev)))
    gid, slot = [], []
    rmax = 0
    for g, rows in enumerate(rows_of_group):
        for k in range(rows):
            gid.append(g)
            slot.append(k)
        rmax = max(rmax, rows)
    return gsum, (torch.as_tensor(gid, dtype=torch.long, device=dev),
                  torch.as_tensor(slot, dtype=torch.long, device=dev)), rmax


def _device_tables(plan, Q, ss, la):
    """Per-device constant tables of a plan (built on first use, reused by every rebuild):
    the Van Loan path arrays of all intervals (one itr_vanloan_paths call per rebuild: jobs
    0 .. I-1 the Van Loan paths of interval i, jobs I .. 2I-1 the interval propagator
    expm(Q dt_i) as a length-1 path), the omega mask rows and every row index as device
    tensors."""
    import torch
    masks = ss.omega_masks
    key = (str(la.dev), tuple(masks))
    if key in plan.dev:
        return plan.dev[key]
    dev = la.dev
    n = Q.shape[0]
    keys = list(masks)
    mid = {k: i for i, k in enumerate(keys)}
    I = len(plan.intervals)
    job, lens, pm = [], [], []
    ivs = []
    for i, ip in enumerate(plan.intervals):
        d = _DevInterval()
        d.vl0 = len(job)
        for p in ip.vl_paths:
            job.append(i)
            lens.append(len(p))
            pm.extend(mid[w] for w in p)
        d.vl1 = len(job)
        ivs.append(d)
    for i, d in enumerate(ivs):
        d.e_idx = len(job)
        job.append(I + i)
        lens.append(1)
        pm.append(0)
    off = np.zeros(len(job) + 1, dtype=np.int64)
    np.cumsum(lens, out=off[1:])
    T = lambda a: torch.as_tensor(np.asarray(a, dtype=np.int64), device=dev)  # noqa: E731
    T32 = lambda a: torch.as_tensor(np.asarray(a, dtype=np.int32), device=dev)  # noqa: E731

    def rows_table(ng, rmax, gid, slot, cols):
        """itr_chain_rows entry tables: [ng * rmax] int32, -1 padding."""
        out = []
        for c in cols:
            t = np.full(ng * rmax, -1, dtype=np.int32)
            if c is not None:
                t[np.asarray(gid) * rmax + np.asarray(slot)] = c
            out.append(T32(t) if c is not None else None)
        return (*out, ng, rmax)

    for d, ip in zip(ivs, plan.intervals):
        src, oms, ome, dst = ip.plain
        d.plain = rows_table(1, src.size, np.zeros(src.size, np.int64), np.arange(src.size),
                             (src, oms, ome, dst)) if src.size else None
        d.ng = len(ip.groups)
        pids_list = [g[0] for g in ip.groups]
        d.sum_steps, (gid, slot), d.rmax = _group_tables(dev, pids_list,
                                                         [g[1].size for g in ip.groups])
        if d.ng:
            cat = lambda j: np.concatenate([g[j] for g in ip.groups])  # noqa: E731
            d.rows = rows_table(d.ng, d.rmax, gid.cpu().numpy(), slot.cpu().numpy(),
                                (cat(1), cat(2), cat(3), cat(4)))
        else:
            d.rows = None
    tab = {
        "mask_u8": np.stack([np.asarray(masks[k], dtype=np.uint8) for k in keys]),
        "job": np.asarray(job, dtype=np.int32), "off": off,
        "pm": np.asarray(pm, dtype=np.int32), "ivs": ivs,
        "F": torch.as_tensor(np.stack([masks[om].astype(np.float64) for om in plan.omegas])
                             if plan.omegas else np.zeros((0, n)), device=dev),
    }
    absorbing = (7, 7)
    keep = ~masks[absorbing]
    tab["keep"] = torch.as_tensor(np.nonzero(keep)[0], dtype=torch.long, device=dev)
    tab["sum_rows"] = T(plan.close_sum_rows)
    cpids = [g[0] for g in plan.close_groups]
    tab["c_steps"], (cg, cs), tab["c_rmax"] = _group_tables(
        dev, cpids, [g[2].size for g in plan.close_groups])
    if plan.close_groups:
        rws = np.concatenate([g[2] for g in plan.close_groups])
        tasks = np.concatenate([g[1] for g in plan.close_groups])
        tab["c_rows"] = rows_table(len(plan.close_groups), tab["c_rmax"], cg.cpu().numpy(),
                                   cs.cpu().numpy(), (rws, None, None, tasks))
    tab["keep32"] = T32(np.nonzero(keep)[0])
    tab["ntasks"] = sum(len(t) for _, t, _ in plan.close_groups)
    plan.dev[key] = tab
    return tab


def _group_matrices(S, gsum, ng, n):
    """M[g] = S[p_g0] + S[p_g1] + ... in path order (see _group_tables); groups g >= gsum.ng
    (padding slots) are zero.  On the device one itr_group_sum launch."""
    import torch
    if S.is_cuda:
        from ..dense import group_sum
        M = (torch.zeros if ng > gsum.ng else torch.empty)((ng, n, n), dtype=S.dtype,
                                                           device=S.device)
        group_sum(S, gsum.off, gsum.paths, gsum.ng, out=M[:gsum.ng])
        return M
    M = torch.zeros((ng, n, n), dtype=S.dtype, device=S.device)
    for gs, ps in gsum.steps:
        M[gs] += S[ps]
    return M


def _unit_members(plan, tab, unit):
    """The members (distinct (interval, sub-path) of length >= 2, vanloan.hip) a unit's paths
    need; a propagator unit needs only its interval's root."""
    i, g = unit
    if g < 0:
        return [((i,), 1)]
    d = tab["ivs"][i]
    off, pm = tab["off"], tab["pm"]
    out = []
    for pid in plan.intervals[i].groups[g][0]:
        p = d.vl0 + int(pid)
        w = tuple(int(x) for x in pm[off[p]:off[p + 1]])
        for x in range(len(w)):
            for y in range(x + 1, len(w)):
                out.append(((i,) + w[x:y + 1], y + 1 - x))
    return out


def split_partition(plan, tab, world):
    """Balanced partition of one rebuild's Van Loan work over `world` ranks.

    Units are an interval's propagator expm(Q dt_i) and each of its path groups (the paths
    one group matrix M_g = S_p0 + S_p1 + ... sums; groups share no path).  A rank's cost is
    the distinct sub-paths ("members", vanloan.hip) its units need, each weighted by its
    length (a member of length k is formed from k - 1 split products at every Pade step);
    members shared by groups of one interval are formed once per rank that needs them.
    Units go interval by interval (groups through the same inner omega pair adjacent) and
    are cut into at most `world`
    contiguous runs: the smallest per-rank cost bound T for which a greedy fill needs no more
    than `world` runs (bisection on T).  Returns per rank (units, cost); unit = (interval,
    -1 for the propagator or the group index)."""
    off, pm = tab["off"], tab["pm"]

    def first_path(i, g):
        d = tab["ivs"][i]
        return min(tuple(int(x) for x in pm[off[d.vl0 + int(p)]:off[d.vl0 + int(p) + 1]])
                   for p in plan.intervals[i].groups[g][0])

    units = []
    for i, d in enumerate(tab["ivs"]):
        units.append((i, -1))
        # groups whose paths pass through the same inner omega pair share most members:
        # keep them adjacent (at 8 ranks of the (7,7) chain: 1.23x instead of 1.33x the
        # ideal per-rank cost)
        fp = {g: first_path(i, g) for g in range(d.ng)}
        units.extend((i, g) for g in sorted(range(d.ng), key=lambda g: (fp[g][1:3], fp[g])))
    mem = [_unit_members(plan, tab, u) for u in units]

    def fill(T):
        runs, cur, seen, c = [], [], set(), 0.0
        for u, ms in zip(units, mem):
            inc = sum(w for k, w in set(ms) if k not in seen)
            if cur and c + inc > T:
                runs.append((cur, c))
                cur, seen, c = [], set(), 0.0
                inc = sum(w for k, w in set(ms))
            cur.append(u)
            seen.update(k for k, _ in ms)
            c += inc
        if cur:
            runs.append((cur, c))
        return runs

    hi_runs = fill(float("inf"))
    lo, hi = hi_runs[0][1] / max(world, 1), hi_runs[0][1]
    best = hi_runs
    for _ in range(40):
        mid = 0.5 * (lo + hi)
        runs = fill(mid)
        if len(runs) <= world:
            best, hi = runs, mid
        else:
            lo = mid
    return best + [([], 0.0)] * (world - len(best))


def _interval_mats_split(plan, tab, Q, t, la):
    """(E_i, M_i) of every interval with the Van Loan work divided over the ranks of
    la.group (split_partition: propagators and path groups cut into runs of equal member
    cost).  Each rank evaluates its units' paths in one itr_vanloan_paths_ex call — every
    interval's Pade branch and scaling taken from the norms of ALL its paths, so each path's
    result is the single-rank one — and forms its group sums in path order; one all-gather
    of the zero-padded unit slots shares them.  The result is bit-identical to world = 1."""
    import torch
    import torch.distributed as dist
    rank, world = la.rank, la.world
    n = Q.shape[0]
    ivs = tab["ivs"]
    I = len(ivs)
    key = ("split", world)
    if key not in tab:
        parts = split_partition(plan, tab, world)
        per_rank = []
        for units, _ in parts:
            job, off0, pm, steps = [], [0], [], []
            for i, g in units:
                d = ivs[i]
                ps = [d.e_idx] if g < 0 else [d.vl0 + int(x) for x in plan.intervals[i].groups[g][0]]
                loc = []
                for p in ps:
                    loc.append(len(job))
                    job.append(int(tab["job"][p]))
                    off0.append(off0[-1] + int(tab["off"][p + 1] - tab["off"][p]))
                    pm.extend(tab["pm"][tab["off"][p]:tab["off"][p + 1]].tolist())
                steps.append(loc)
            per_rank.append((units, np.asarray(job, dtype=np.int32),
                             np.asarray(off0, dtype=np.int64), np.asarray(pm, dtype=np.int32),
                             _group_tables(la.dev, steps, [0] * len(steps))[0]))
        tab[key] = ([c for _, c in parts], per_rank)
    _, per_rank = tab[key]
    units, job, off0, pm, steps = per_rank[rank]
    slots = max(len(u[0]) for u in per_rank)
    if units:
        norms = la.vanloan_norms(Q, tab["mask_u8"], t, tab["job"], tab["off"], tab["pm"])
        S = la.vanloan_batch(Q, tab["mask_u8"], t, job, off0, pm, job_norm=norms)
        # slot k = M_g = S_p0 + S_p1 + ... in path order (a propagator: its S)
        buf = _group_matrices(S, steps, slots, n)
    else:
        buf = torch.zeros((slots, n, n), dtype=torch.float64, device=la.dev)
    if buf.is_cuda and dist.get_backend(la.group) != "nccl":
        buf = buf.cpu()  # gloo rehearsal of the exchange (tests: ranks sharing one GPU)
    got = [torch.empty_like(buf) for _ in range(world)]
    dist.all_gather(got, buf, group=la.group)
    got = [x.to(la.dev) for x in got]
    E = [None] * I
    M = [[None] * d.ng for d in ivs]
    for r, pr in enumerate(per_rank):
        for k, (i, g) in enumerate(pr[0]):
            if g < 0:
                E[i] = got[r][k]
            else:
                M[i][g] = got[r][k]
    return [(E[i], torch.stack(M[i]) if ivs[i].ng else None) for i in range(I)]


def _run_chain_abc_device(plan, Q, times, ss, probs: Dict, la) -> Dict:
    """_run_chain_abc_planned with every number resident on the device: one shared Van Loan
    evaluation for all intervals (their propagators included), the key rows as one
    [rows, n] tensor advanced interval by interval, the closing phase's contractions; a
    single device-to-host copy of the final per-key probabilities."""
    import torch
    from ..dense import h2d
    tab = _device_tables(plan, Q, ss, la)
    masks = ss.omega_masks
    n = Q.shape[0]
    dev = la.dev
    I = len(plan.intervals)
    t = np.asarray([times[i] for i in range(I)] * 2, dtype=np.float64)
    if getattr(la, "world", 1) > 1:
        EM = _interval_mats_split(plan, tab, Q, t, la)
    else:
        S_all = _take_prefetch(plan, Q, t, la)
        if S_all is None:
            S_all = la.vanloan_batch(Q, tab["mask_u8"], t, tab["job"], tab["off"], tab["pm"])
        EM = [(S_all[d.e_idx],
               _group_matrices(S_all[d.vl0:d.vl1], d.sum_steps, d.ng, n) if d.ng else None)
              for d in tab["ivs"]]
    F = tab["F"]
    P = torch.zeros((plan.nrows, n), dtype=torch.float64, device=dev)
    P0 = np.zeros((len(probs), n))
    for i, v in enumerate(probs.values()):
        P0[i] = v[0]
    P[:len(probs)] = h2d(P0) if P.is_cuda else torch.from_numpy(P0)
    for d, (E, M) in zip(tab["ivs"], EM):
        # (P * mask) @ propagator * mask for every key row of the interval, gathered, multiplied
        # and scattered by one fused kernel per matrix kind (itr_chain_rows)
        Pn = P.clone()
        if d.plain is not None:
            la.chain_rows(P, F, E.contiguous(), d.plain, Pn)
        if d.rows is not None:
            la.chain_rows(P, F, M.contiguous(), d.rows, Pn)
        P = Pn
    absorbing = (7, 7)
    keep = tab["keep"]
    Qn = Q[~masks[absorbing]][:, ~masks[absorbing]]
    sums = P[tab["sum_rows"]].sum(dim=1) if plan.close_sum_rows.size else \
        torch.zeros(0, dtype=torch.float64, device=dev)
    deep = torch.zeros(tab["ntasks"], dtype=torch.float64, device=dev)
    if plan.close_paths:
        D = la.deepest_t(Qn, masks_without(masks, absorbing), plan.close_paths)
        ng = len(plan.close_groups)
        nk = keep.numel()
        M = _group_matrices(D, tab["c_steps"], ng, nk)
        R = torch.zeros((tab["ntasks"], nk), dtype=torch.float64, device=dev)
        la.chain_rows(P, None, M.contiguous(), tab["c_rows"], R, cols=tab["keep32"])
        deep = R.sum(dim=1)
    host = torch.cat([sums, deep]).cpu().numpy()
    ns = sums.numel()
    out: Dict = {}
    for key, kind, k in plan.close_order:
        out[key] = float(host[k]) if kind == "sum" else float(host[ns + k])
    return out


def _products_in_order(plan, probs, E, vl_needed, fmask) -> None:
    """run_markov_chain_ABC.py:407-490 path by path (reads see earlier writes)."""
    for path, plain, vl in plan:
        pm = probs[path]
        writes = []
        for key, om_s, om_e in plain:
            writes.append((key, (pm * fmask[om_s]) @ E * fmask[om_e]))
        for key6, sub, om_s, om_e in vl:
            S = vl_needed[sub[0]].copy()
            for p in sub[1:]:
                S = S + vl_needed[p]
            writes.append(((key6[:3], key6[3:]), (pm * fmask[om_s]) @ S * fmask[om_e]))
        for key, v in writes:  # plain results first, then Van Loan ones
            probs[key] = v


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


def _expm2(Q, t):
    """expm(Q t) of a two-state rate matrix [[-a, a], [b, -b]] in closed form:
    (1/s) [[b + a e, a (1 - e)], [b (1 - e), a + b e]] with s = a + b, e = e^{-s t} (within a
    few ulp of expm.py's Pade evaluation, get_joint_prob_mat.py:119-123; no device round trip
    for three 2 x 2 matrices)."""
    a, b = Q[0, 1], Q[1, 0]
    sr = a + b
    if sr == 0.0:
        return np.eye(2)
    om = -np.expm1(-sr * t)  # 1 - e
    e = 1.0 - om
    return np.array([[b + a * e, a * om], [b * om, a + b * e]]) / sr


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
    Ea, Eb, Ec = (_expm2(Qa, t_A), _expm2(Qb, t_B), _expm2(Qc, t_C))
    fa = (pi1 @ Ea).reshape(1, -1)
    fb = (pi1 @ Eb).reshape(1, -1)
    fc = (pi1 @ Ec).reshape(1, -1)
    pi_ab = {START: combine_states(s1, s1, s2, fa, fb)}
    ab = run_chain_ab(Qab, _interval_lengths(cut_AB), s2.omega_masks, pi_ab, n_int_AB, la)
    pi_abc = {path: combine_states(s2, s1, s3, p, fc) for path, p in ab.items()}
    return run_chain_abc(Qabc, _interval_lengths(cut_ABC), s3, pi_abc, n_int_ABC, la)
