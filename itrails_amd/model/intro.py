"""trans_emiss_calc_introgression (int_get_trans_emiss.py:9-185): the HMM (a, b, pi) of the
iTRAILS model with introgression from the C lineage into B.

The reference builds it in three stages, restated here in the same order:

1. One- and two-sequence chains up to the second speciation (int_get_joint_prob_mat.py:16-263,
   int_get_tab.py:17-812): species A, B, C one-sequence chains; B split by the admixture
   proportion m into a "left" path (stays with A) and a "right" path (migrates to C); the AB
   and BC two-sequence chains (full, and with one B lineage missing) run over the AB
   intervals and are mixed into one 203-state start vector of the three-sequence chain per
   two-site fate (deep / V0 / introgressed, per interval) — `_ab_table`.
2. The three-sequence chain over the ABC intervals (int_get_tab.py:815-1500, get_tab.py:
   713-1301): every pair of hidden states (topology, first interval, second interval) gets
   pi @ (product of propagators restricted to state classes) summed — `_abc_table`.  Every
   heavy factor (interval propagators expm(Q t), Van Loan block exponentials, the inverse
   blocks of the open last interval) is planned first, de-duplicated and evaluated as
   batches on the device (`la.expm`, `la.vanloan`, `la.deepest`: dense.hip); the host then
   only multiplies row vectors through the restricted matrices.
3. Emissions (int_get_emission_prob_mat.py:744-1110): the reference's single/double
   coalescence emission functions are the plain model's (identical code), only the per-state
   branch times differ — `int_state_specs` feeds emissions.emission_rows (emission.hip).

Hidden states are (topology, i, j): 0 = V0 (A, B coalesce in AB interval i), 4 = the
introgressed V0 (B, C coalesce in BC interval i), 1-3 = deep coalescence (ILS topologies);
sorted by tuple like the reference's pandas pivot (int_get_trans_emiss.py:133-140).

State spaces.  The reference reads the CTMC state spaces from package CSV files
(int_load_trans_mat.py:6-41).  A state is a set of lineage blocks (left-site species mask,
right-site species mask); the CSV chains are exactly "merge any two blocks at rate C" and
"split a block that carries both sites at rate R" (checked transition by transition against
load_trans_mat in tests/test_intro_host.py), so they are generated here.  The state order
inside the two- and three-sequence chains is internal to the computation (every quantity is
addressed by state content), except that the reference drops the last two (absorbing)
three-sequence states for the open interval (int_get_tab.py:1361) and addresses the
one-sequence chain by position; both conventions are kept.
"""
from __future__ import annotations

import itertools
from functools import lru_cache
from typing import Dict, List, Sequence, Tuple

import numpy as np
from scipy.special import comb

from .emissions import branch_generator, cutpoints_AB, cutpoints_ABC, emission_rows
from .trans_emiss import OBSERVED_NAMES

State = Tuple[Tuple[int, int], ...]   # sorted blocks (left mask, right mask)

# ---------------------------------------------------------------------------------------
# state spaces and rate matrices
# ---------------------------------------------------------------------------------------


def _moves(st: State):
    """(target, symbol) of every transition out of `st`: C merges two blocks, R splits a
    block that carries lineages of both sites."""
    out = []
    for i, j in itertools.combinations(range(len(st)), 2):
        a, b = st[i], st[j]
        rest = [x for k, x in enumerate(st) if k not in (i, j)]
        out.append((tuple(sorted(rest + [(a[0] | b[0], a[1] | b[1])])), "C"))
    for i, a in enumerate(st):
        if a[0] and a[1]:
            rest = [x for k, x in enumerate(st) if k != i]
            out.append((tuple(sorted(rest + [(a[0], 0), (0, a[1])])), "R"))
    return out


def chain_states(masks: Sequence[int]) -> List[State]:
    """All states reachable from the fully unlinked, uncoalesced state of the species
    `masks`; breadth-first, the two all-coalesced (absorbing) states last."""
    start = tuple(sorted([(0, s) for s in masks] + [(s, 0) for s in masks]))
    seen, order, k = {start}, [start], 0
    while k < len(order):
        for t, _ in _moves(order[k]):
            if t not in seen:
                seen.add(t)
                order.append(t)
        k += 1
    full = 0
    for s in masks:
        full |= s
    last = [((0, full), (full, 0)), ((full, full),)]
    return [s for s in order if s not in last] + [s for s in last if s in seen]


def symbols(states: Sequence[State]) -> np.ndarray:
    """The 'R' / 'C' / '0' matrix of load_trans_mat (int_load_trans_mat.py:6-41)."""
    idx = {s: i for i, s in enumerate(states)}
    m = np.full((len(states), len(states)), "0", dtype=object)
    for i, s in enumerate(states):
        for t, v in _moves(s):
            if t in idx:
                m[i, idx[t]] = v
    return m


def rate_matrix(sym: np.ndarray, coal: float, rho: float) -> np.ndarray:
    """trans_mat_num (int_load_trans_mat.py:44-84): C -> coal, R -> rho, diagonal -row sum."""
    n = sym.shape[0]
    q = np.zeros((n, n))
    for i in range(n):
        for j in range(n):
            if sym[i, j] != "0":
                q[i, j] = coal if sym[i, j] == "C" else rho
    for i in range(n):
        q[i, i] = -sum(q[i])
    return q


# one-sequence chain in the reference's CSV order: linked first (int_get_joint_prob_mat.py
# uses row 0 as the start and entry 1 as "unlinked", :133-145, 266-303)
def one_seq(mask: int) -> List[State]:
    return [((mask, mask),), ((0, mask), (mask, 0))]


# the chain of one missing B lineage (load_trans_mat_miss, int_get_joint_prob_mat.py:306-339):
# states 0-4 hold B's left-site lineage, 5-9 its right-site lineage, with both sites of C
MISS_BC: List[State] = [
    ((2, 0), (4, 4)), ((0, 4), (2, 0), (4, 0)), ((2, 4), (4, 0)), ((0, 4), (6, 0)), ((6, 4),),
    ((0, 2), (4, 4)), ((0, 2), (0, 4), (4, 0)), ((0, 4), (4, 2)), ((0, 6), (4, 0)), ((4, 6),),
]


def _relabel(st: State, mp: Dict[int, int]) -> State:
    return tuple(sorted((mp.get(l, l), mp.get(r, r)) for l, r in st))


def _values(st: State):
    """(left values, right values) of the flattened state (`flatten[i][::2]`, `[1::2]`)."""
    return [b[0] for b in st], [b[1] for b in st]


# ---------------------------------------------------------------------------------------
# stage 1: chains up to the second speciation (get_tab_AB_introgression)
# ---------------------------------------------------------------------------------------


def _combine(sa, sb, pa, pb, acc: Dict[State, float]):
    """combine_states (int_combine_states.py:4-44) accumulated into `acc` in call order."""
    part: Dict[State, float] = {}
    for i in range(len(sa)):
        for j in range(len(sb)):
            k = tuple(sorted(sa[i] + sb[j]))
            part[k] = part.get(k, 0.0) + pa[i] * pb[j]
    for k in sorted(part, key=lambda s: str([tuple(b) for b in s])):
        acc[k] = acc.get(k, 0.0) + part[k]


class _Chain2:
    """A two-sequence chain over the AB (or BC) intervals: states, the interval
    propagators and its start vector; `final(...)` is pi @ get_AB_precomp ordered back to
    the full state list (int_get_tab.py:150-160, get_tab.py:35-54, int_get_ordered.py)."""

    def __init__(self, states, P, pi, marker):
        self.states, self.P, self.pi = states, P, np.asarray(pi, dtype=np.float64)
        n = len(states)
        self.tot = list(range(n))
        lv = [_values(s) for s in states]
        self.cls = {
            "tot": self.tot,
            "B": [i for i in range(n) if marker not in lv[i][0] + lv[i][1]],
            "L": [i for i in range(n) if marker in lv[i][0] and marker not in lv[i][1]],
            "R": [i for i in range(n) if marker not in lv[i][0] and marker in lv[i][1]],
            "E": [i for i in range(n) if marker in lv[i][0] and marker in lv[i][1]],
        }

    def final(self, seq: Sequence[str]) -> np.ndarray:
        om = [self.cls[c] for c in ["tot"] + list(seq)]
        v = self.pi
        for k in range(len(self.P)):
            v = v @ self.P[k][np.ix_(om[k], om[k + 1])]
        out = np.zeros(len(self.states))
        out[om[-1]] = v
        return out

    def zeros(self) -> np.ndarray:
        return np.zeros(len(self.states))


def _ab_table(n_ab, ch, sp_abc, final_A_bis, final_C_bis, pi_ABm, pi_BCm):
    """Rows of start vectors of the three-sequence chain, one per two-site fate, in the
    order of get_tab_AB_introgression (int_get_tab.py:132-812)."""
    ABf, ABm, BCf, BCm = ch["ABf"], ch["ABm"], ch["BCf"], ch["BCm"]
    A_sp, C_sp = one_seq(1), one_seq(4)
    abc_index = {s: i for i, s in enumerate(sp_abc)}
    sABm0, sABm1 = sum(pi_ABm[5:]), sum(pi_ABm[0:5])
    sBCm0, sBCm1 = sum(pi_BCm[0:5]), sum(pi_BCm[5:])

    def mix(f_ABm, f_BCm, f_ABf, f_BCf):  # mix_probs (int_get_tab.py:17-129)
        acc: Dict[State, float] = {}
        _combine(ABm.states[5:], BCm.states[0:5], f_ABm[5:], f_BCm[0:5] / sBCm0, acc)
        _combine(ABm.states[5:], BCm.states[0:5], f_ABm[5:] / sABm0, f_BCm[0:5], acc)
        _combine(ABm.states[0:5], BCm.states[5:], f_ABm[0:5], f_BCm[5:] / sBCm1, acc)
        _combine(ABm.states[0:5], BCm.states[5:], f_ABm[0:5] / sABm1, f_BCm[5:], acc)
        _combine(ABf.states, C_sp, f_ABf, final_C_bis, acc)
        _combine(BCf.states, A_sp, f_BCf, final_A_bis, acc)
        row = np.zeros(len(sp_abc))
        for k, v in acc.items():
            row[abc_index[k]] = v
        return row

    n = n_ab
    rows, names = [], []

    def dseq():
        return ["B"] * n

    def one(side, x):  # [B]*x + [side]*(n-x), ordered by `side`
        return ["B"] * x + [side] * (n - x)

    def two(L, R):  # both sites coalesced (int_get_tab.py:509-533)
        if R == L:
            return ["B"] * L + ["E"] * (n - L)
        if L < R:
            return ["B"] * L + ["L"] * (R - L) + ["E"] * (n - R)
        return ["B"] * R + ["R"] * (L - R) + ["E"] * (n - L)

    # deep -> deep
    rows.append(mix(ABm.final(dseq()), BCm.final(dseq()), ABf.final(dseq()), BCf.final(dseq())))
    names.append(("D", "D"))
    # V0 -> deep, deep -> V0
    bcm_d = BCm.final(dseq())
    for L in range(n):
        rows.append(mix(ABm.final(one("L", L)), bcm_d, ABf.final(one("L", L)), BCf.zeros()))
        names.append(((0, L), "D"))
    for R in range(n):
        rows.append(mix(ABm.final(one("R", R)), bcm_d, ABf.final(one("R", R)), BCf.zeros()))
        names.append(("D", (0, R)))
    # introgression -> deep, deep -> introgression
    abm_d = ABm.final(dseq())
    for L in range(n):
        rows.append(mix(abm_d, BCm.final(one("L", L)), ABf.zeros(), BCf.final(one("L", L))))
        names.append(((4, L), "D"))
    for R in range(n):
        rows.append(mix(abm_d, BCm.final(one("R", R)), ABf.zeros(), BCf.final(one("R", R))))
        names.append(("D", (4, R)))
    # V0 -> V0
    for L in range(n):
        for R in range(n):
            rows.append(mix(ABm.zeros(), BCm.zeros(), ABf.final(two(L, R)), BCf.zeros()))
            names.append(((0, L), (0, R)))
    # introgression -> introgression
    for L in range(n):
        for R in range(n):
            rows.append(mix(ABm.zeros(), BCm.zeros(), ABf.zeros(), BCf.final(two(L, R))))
            names.append(((4, L), (4, R)))
    # V0 -> introgression, introgression -> V0
    for L in range(n):
        for R in range(n):
            rows.append(mix(ABm.final(one("L", L)), BCm.final(one("R", R)), ABf.zeros(),
                            BCf.zeros()))
            names.append(((0, L), (4, R)))
    for L in range(n):
        for R in range(n):
            rows.append(mix(ABm.final(one("R", R)), BCm.final(one("L", L)), ABf.zeros(),
                            BCf.zeros()))
            names.append(((4, L), (0, R)))
    return np.array(rows), names


def _split_migration(sp: List[State], p: np.ndarray, m: float, direction: str):
    """split_migration (int_get_joint_prob_mat.py:266-303)."""
    x = p[1]
    st = [sp[0], sp[1], (sp[1][0],), (sp[1][1],)]
    if direction == "left":
        pr = np.array([(1 - x) * (1 - m), (1 - m) ** 2 * x, 1 / 2 * (1 - m) * m * x,
                       1 / 2 * (1 - m) * m * x])
    else:
        pr = np.array([(1 - x) * m, x * m ** 2, 1 / 2 * (1 - m) * m * x,
                       1 / 2 * (1 - m) * m * x])
    return st, pr


def _ordered_start(sa, sb, pa, pb, space):
    """combine_states then re-ordered by `space` (int_get_joint_prob_mat.py:165-169)."""
    acc: Dict[State, float] = {}
    _combine(sa, sb, pa, pb, acc)
    return [acc.get(s, 0) for s in space]


# ---------------------------------------------------------------------------------------
# stage 2: the three-sequence chain (get_tab_ABC_introgression, pool_AB_total, pool_ABC)
# ---------------------------------------------------------------------------------------
_NUM = {3: 1, 5: 2, 6: 3}   # dct_num: coalesced pair -> deep topology


def abc_classes(states: Sequence[State]) -> Dict[str, List[int]]:
    """om (int_get_tab.py:842-876): states by (left, right) coalescence class."""
    om: Dict[str, List[int]] = {}
    lv = [_values(s) for s in states]
    n = len(states)
    ks = [3, 5, 6, 7]
    for l in [0, 3, 5, 6, 7]:
        for r in [0, 3, 5, 6, 7]:
            if l in ks and r in ks:
                om[f"{l}{r}"] = [i for i in range(n) if l in lv[i][0] and r in lv[i][1]]
            elif l == 0 and r in ks:
                om[f"{l}{r}"] = [i for i in range(n) if all(x not in ks for x in lv[i][0])
                                 and r in lv[i][1]]
            elif l in ks and r == 0:
                om[f"{l}{r}"] = [i for i in range(n) if l in lv[i][0]
                                 and all(x not in ks for x in lv[i][1])]
            else:
                om[f"{l}{r}"] = [i for i in range(n)
                                 if all(x not in ks for x in lv[i][0] + lv[i][1])]
    om["71"] = sorted(om["73"] + om["75"] + om["76"])
    om["17"] = sorted(om["37"] + om["57"] + om["67"])
    om["10"] = sorted(om["30"] + om["50"] + om["60"])
    om["13"] = sorted(om["33"] + om["53"] + om["63"])
    om["15"] = sorted(om["35"] + om["55"] + om["65"])
    om["16"] = sorted(om["36"] + om["56"] + om["66"])
    om["11"] = sorted(om["13"] + om["15"] + om["16"])
    om["tot"] = list(range(n))
    return om


class _ABCPlan:
    """Table entries of the three-sequence stage as sums of row-vector chains.

    A chain is a list of factors, each a restricted matrix M[rows][:, cols] with rows/cols
    given as class names:
      ("P", k, r, c)         interval propagator expm(Q t_k)         (get_tab.py:17-33, 57-82)
      ("S", r, c)            identity (get_ABC_precomp with no interval, get_tab.py:75-77)
      ("VL", path, k, r, c)  expm(C t_k)[:n, -n:], C = Van Loan blocks over `path`
                             (int_vanloan.py:34-132)
      ("INF", path, r, c)    (-C^-1)[:n, -n:] @ A_last over the 201 transient states for
                             the open last interval (int_get_tab.py:1361-1408, get_tab.py:850-990)
    An entry's value is sum over its chains of (pi @ chain).sum().
    """

    def __init__(self, cut_ABC):
        self.cut = cut_ABC
        self.n = len(cut_ABC) - 1
        self.entries: Dict[Tuple, Tuple[str, List[list]]] = {}
        self.order: List[Tuple] = []

    def fin(self, k):  # cut_ABC[k + 1] != inf
        return int(self.cut[k + 1] != np.inf)

    def pre(self, omegas, idx):
        """get_ABC_precomp(pr, omegas, idx_lst) (get_tab.py:57-82)."""
        if len(idx) == 0:
            return [("S", omegas[0], omegas[0])]
        return [("P", idx[i], omegas[i], omegas[i + 1]) for i in range(len(idx))]

    def add(self, src, dst, pi_name, chains):
        key = (src, dst)
        if key in self.entries:
            raise ValueError(f"duplicate joint entry {key}")
        self.entries[key] = (pi_name, chains)
        self.order.append(key)

    def add_sym(self, src, dst, pi_name, chains):
        self.add(src, dst, pi_name, chains)
        self.add(dst, src, pi_name, chains)


def _plan_v0_i(P: _ABCPlan, n_ab):
    """V0 -> V0, I -> I, V0 -> I, I -> V0 (int_get_tab.py:896-1072)."""
    n = P.n
    for a, b in ((0, 0), (4, 4)):
        for l in range(n_ab):
            for r in range(n_ab):
                pn = ((a, l), (b, r))
                for L in range(n):
                    for R in range(n):
                        if L < R:
                            om = ["tot"] + ["11"] * L + ["71"] * (R - L) + ["77"]
                            ch = P.pre(om, list(range(R + P.fin(R))))
                            P.add_sym((a, l, L), (b, r, R), pn, [ch])
                        elif L == R:
                            om = ["tot"] + ["11"] * L + ["77"]
                            P.add((a, l, L), (b, r, R), pn, [P.pre(om, list(range(L + P.fin(L))))])
    for a, b in ((0, 4), (4, 0)):
        for l in range(n_ab):
            for r in range(n_ab):
                pn = ((a, l), (b, r))
                for L in range(n):
                    for R in range(n):
                        if L < R:
                            om = ["tot"] + ["11"] * L + ["71"] * (R - L) + ["77"]
                            ch = P.pre(om, list(range(R + P.fin(R))))
                        elif L > R:
                            om = ["tot"] + ["11"] * R + ["17"] * (L - R) + ["77"]
                            ch = P.pre(om, list(range(L + P.fin(L))))
                        else:
                            om = ["tot"] + ["11"] * L + ["77"]
                            ch = P.pre(om, list(range(L + P.fin(L))))
                        P.add((a, l, L), (b, r, R), pn, [ch])


def _plan_ab_total(P: _ABCPlan, n_ab, L, r, R):
    """pool_AB_total (int_get_tab.py:1230-1500): V0/I -> deep and deep -> V0/I."""
    fin = P.fin

    def emit(i, chains):
        ii = _NUM[i]
        for l in range(n_ab):
            for a in (0, 4):
                P.add_sym((a, l, L), (ii, r, R), ((a, l), "D"), chains)

    if L < r < R:
        pre = ["tot"] + ["10"] * L + ["70"] * (r - L)
        for i in (3, 5, 6):
            om = pre + [f"7{i}"] * (R - r) + ["77"]
            emit(i, [P.pre(om, list(range(R + fin(R))))])
    elif L == r < R:
        pre = ["tot"] + ["10"] * L
        for i in (3, 5, 6):
            om = pre + [f"7{i}"] * (R - L) + ["77"]
            emit(i, [P.pre(om, list(range(R + fin(R))))])
    elif r < L < R:
        pre = ["tot"] + ["10"] * r
        for i in (3, 5, 6):
            om = pre + [f"1{i}"] * (L - r) + [f"7{i}"] * (R - L) + ["77"]
            emit(i, [P.pre(om, list(range(R + fin(R))))])
    elif r < L == R:
        pre = ["tot"] + ["10"] * r
        for i in (3, 5, 6):
            om = pre + [f"1{i}"] * (L - r) + ["77"]
            emit(i, [P.pre(om, list(range(R + fin(R))))])
    elif r < R < L:
        pre = ["tot"] + ["10"] * r
        for i in (3, 5, 6):
            om = pre + [f"1{i}"] * (R - r) + ["17"] * (L - R) + ["77"]
            emit(i, [P.pre(om, list(range(L + fin(L))))])
    elif L < r == R:
        base = P.pre(["tot"] + ["10"] * L + ["70"] * (r - L), list(range(R)))
        for i in (3, 5, 6):
            if fin(r):
                res = ("VL", ("70", f"7{i}"), r, "70", "77")
            else:
                res = ("INF", ("70", f"7{i}"), "70", f"7{i}")
            emit(i, [base + [res]])
    elif L == r == R:
        pre = P.pre(["tot"] + ["10"] * R, list(range(R)))
        start = [("S", "tot", "10")] if L == 0 else pre
        for i in (3, 5, 6):
            if not fin(r):
                chains = [start + [("INF", ("10", f"1{i}"), "10", f"1{i}")],
                          start + [("INF", ("10", f"7{i}"), "10", f"7{i}")],
                          start + [("INF", ("10", "70", f"7{i}"), "10", f"7{i}")]]
            else:
                lst = ["10", f"1{i}", "17", "70", f"7{i}", "77"]
                chains = []
                for y in range(1, len(lst)):
                    for z in range(y + 1, len(lst)):
                        if int(lst[z][0]) < int(lst[y][0]):
                            continue
                        if int(lst[z][1]) < int(lst[y][1]):
                            continue
                        if int(lst[z][1]) - int(lst[y][1]) == 7:
                            continue
                        if lst[y][1] == "7":
                            continue
                        chains.append(start + [("VL", (lst[0], lst[y], lst[z]), r, "10", "77")])
            emit(i, chains)
    elif r == R < L:
        pre = P.pre(["tot"] + ["10"] * R, list(range(R)))
        start = [("S", "tot", "10")] if R == 0 else pre
        end = P.pre(["17"] * (L - R) + ["77"], list(range(R + 1, L + fin(L))))
        for i in (3, 5, 6):
            emit(i, [start + [("VL", ("10", f"1{i}"), r, "10", "17")] + end])


def _plan_abc_pool(P: _ABCPlan, l, L, r, R):
    """pool_ABC (get_tab.py:713-1301): deep -> deep, pi = the ("D", "D") row."""
    fin = P.fin
    pn = ("D", "D")

    def put(i, j, chains, sym=True):
        a, b = (_NUM[i], l, L), (_NUM[j], r, R)
        (P.add_sym if sym else P.add)(a, b, pn, chains)

    if l < L < r < R:
        for i in (3, 5, 6):
            for j in (3, 5, 6):
                om = (["tot"] + ["00"] * l + [f"{i}0"] * (L - l) + ["70"] * (r - L)
                      + [f"7{j}"] * (R - r) + ["77"])
                put(i, j, [P.pre(om, list(range(R + fin(R))))])
    elif l < L == r < R:
        for i in (3, 5, 6):
            for j in (3, 5, 6):
                om = (["tot"] + ["00"] * l + [f"{i}0"] * (L - l) + [f"7{j}"] * (R - L)
                      + ["77"])
                put(i, j, [P.pre(om, list(range(R + fin(R))))])
    elif l == r < L < R:
        for i in (3, 5, 6):
            for j in (3, 5, 6):
                om = (["tot"] + ["00"] * l + [f"{i}{j}"] * (L - l) + [f"7{j}"] * (R - L)
                      + ["77"])
                put(i, j, [P.pre(om, list(range(R + fin(R))))])
    elif l < r < L < R:
        for i in (3, 5, 6):
            for j in (3, 5, 6):
                om = (["tot"] + ["00"] * l + [f"{i}0"] * (r - l) + [f"{i}{j}"] * (L - r)
                      + [f"7{j}"] * (R - L) + ["77"])
                put(i, j, [P.pre(om, list(range(R + fin(R))))])
    elif r < l < L < R:
        for i in (3, 5, 6):
            for j in (3, 5, 6):
                om = (["tot"] + ["00"] * r + [f"0{j}"] * (l - r) + [f"{i}{j}"] * (L - l)
                      + [f"7{j}"] * (R - L) + ["77"])
                put(i, j, [P.pre(om, list(range(R + fin(R))))])
    elif l == r < L == R:
        for i in (3, 5, 6):
            for j in (3, 5, 6):
                om = ["tot"] + ["00"] * l + [f"{i}{j}"] * (L - l) + ["77"]
                put(i, j, [P.pre(om, list(range(R + fin(R))))], sym=False)
    elif l < r < L == R:
        for i in (3, 5, 6):
            for j in (3, 5, 6):
                om = (["tot"] + ["00"] * l + [f"{i}0"] * (r - l) + [f"{i}{j}"] * (R - r)
                      + ["77"])
                put(i, j, [P.pre(om, list(range(R + fin(R))))])
    elif l == r == L == R:
        pre = P.pre(["tot"] + ["00"] * R, list(range(R)))
        start = [("S", "tot", "00")] if L == 0 else pre
        for i in (3, 5, 6):
            for j in (3, 5, 6):
                ij, i0, j0, i7, j7 = f"{i}{j}", f"{i}0", f"0{j}", f"{i}7", f"7{j}"
                if not fin(r):
                    paths = [(("00", ij), ij), (("00", i0, ij), ij), (("00", j0, ij), ij),
                             (("00", j0, "07", i7), i7), (("00", i0, "70", j7), j7),
                             (("00", j0, i7), i7), (("00", i0, j7), j7)]
                    chains = [start + [("INF", p, "00", c)] for p, c in paths]
                else:
                    tups = [("00", i0, j7, "77"), ("00", j0, i7, "77")]
                    for z in (i7, j7):
                        tups.append(("00", ij, z, "77"))
                    for y in (i0, j0):
                        for z in (ij, "70", "07"):
                            if int(y[0]) - int(z[0]) == -7 or int(y[1]) - int(z[1]) == -7:
                                continue
                            for v in (i7, j7, "77"):
                                if int(z[0]) > int(v[0]) or int(z[1]) > int(v[1]):
                                    continue
                                if int(z[0]) - int(v[0]) == -7 or int(z[1]) - int(v[1]) == -7:
                                    continue
                                tups.append(("00", y, z, v))
                    chains = [start + [("VL", t, r, "00", "77")] for t in tups]
                    chains.append(start + [("VL", ("00", ij, "77"), r, "00", "77")])
                put(i, j, chains, sym=False)
    elif l == L < r == R:
        pre = P.pre(["tot"] + ["00"] * L, list(range(L)))
        start = [("S", "tot", "00")] if L == 0 else pre
        end = P.pre(["70"] * (R - L), list(range(L + 1, R)))
        for i in (3, 5, 6):
            res1 = ("VL", ("00", f"{i}0"), l, "00", "70")
            for j in (3, 5, 6):
                if not fin(r):
                    res2 = ("INF", ("70", f"7{j}"), "70", f"7{j}")
                else:
                    res2 = ("VL", ("70", f"7{j}"), r, "70", "77")
                put(i, j, [start + [res1] + end + [res2]])
    elif l == L < r < R:
        for j in (3, 5, 6):
            pre = P.pre(["tot"] + ["00"] * L, list(range(L)))
            start = [("S", "tot", "00")] if L == 0 else pre
            end = P.pre(["70"] * (r - L) + [f"7{j}"] * (R - r) + ["77"],
                        list(range(L + 1, R + fin(R))))
            for i in (3, 5, 6):
                res = ("VL", ("00", f"{i}0"), l, "00", "70")
                put(i, j, [start + [res] + end])
    elif l == L == r < R:
        pre = P.pre(["tot"] + ["00"] * L, list(range(L)))
        start = [("S", "tot", "00")] if L == 0 else pre
        for j in (3, 5, 6):
            for i in (3, 5, 6):
                end = P.pre([f"7{j}"] * (R - L) + ["77"], list(range(L + 1, R + fin(R))))
                lst = ["00", f"{i}0", f"0{j}", f"{i}{j}", "70", f"7{j}"]
                chains = []
                for y in range(1, len(lst)):
                    for z in range(y + 1, len(lst)):
                        if int(lst[z][0]) < int(lst[y][0]):
                            continue
                        if int(lst[z][1]) < int(lst[y][1]):
                            continue
                        if int(lst[z][0]) - int(lst[y][0]) == 7:
                            continue
                        if lst[y][0] == "7":
                            continue
                        chains.append(start + [("VL", (lst[0], lst[y], lst[z]), r, "00",
                                                f"7{j}")] + end)
                put(i, j, chains)
    elif l < L == r == R:
        for i in (3, 5, 6):
            base = P.pre(["tot"] + ["00"] * l + [f"{i}0"] * (L - l), list(range(L)))
            for j in (3, 5, 6):
                i0 = f"{i}0"
                if not fin(L):
                    chains = [base + [("INF", (i0, f"1{j}"), i0, f"1{j}")],
                              base + [("INF", (i0, f"7{j}"), i0, f"7{j}")],
                              base + [("INF", (i0, "70", f"7{j}"), i0, f"7{j}")]]
                else:
                    lst = [i0, f"{i}{j}", f"{i}7", "70", f"7{j}", "77"]
                    chains = [base + [("VL", (lst[0], lst[y], lst[z]), r, i0, "77")]
                              for y in range(1, len(lst)) for z in range(y + 1, len(lst))]
                put(i, j, chains)
    elif l < L < r == R:
        for i in (3, 5, 6):
            base = P.pre(["tot"] + ["00"] * l + [f"{i}0"] * (L - l) + ["70"] * (r - L),
                         list(range(r)))
            for j in (3, 5, 6):
                if fin(r):
                    res = ("VL", ("70", f"7{j}"), r, "70", "77")
                else:
                    res = ("INF", ("70", f"7{j}"), "70", f"7{j}")
                put(i, j, [base + [res]])
    elif r < l == L < R:
        for j in (3, 5, 6):
            start = P.pre(["tot"] + ["00"] * r + [f"0{j}"] * (l - r), list(range(l)))
            end = P.pre([f"7{j}"] * (R - l) + ["77"], list(range(l + 1, R + fin(R))))
            for i in (3, 5, 6):
                res = ("VL", (f"0{j}", f"{i}{j}"), l, f"0{j}", f"7{j}")
                put(i, j, [start + [res] + end])


def _pool_abc_list(n):
    """The (l, L, r, R) task list of get_tab_ABC_introgression (int_get_tab.py:1161-1197)."""
    out = []
    for l in range(n):
        for L in range(l, n):
            for r in range(n):
                for R in range(r, n):
                    if (l < L < r < R or l < L == r < R or l == r < L < R or l < r < L < R
                            or r < l < L < R or l == r < L == R or l < r < L == R
                            or l == r == L == R or l == L < r == R or l == L < r < R
                            or l == L == r < R or l < L == r == R or l < L < r == R
                            or r < l == L < R):
                        out.append((l, L, r, R))
    return out


def _pool_ab_list(n):
    """The (L, r, R) task list of pool_AB_total (int_get_tab.py:1084-1103)."""
    out = []
    for L in range(n):
        for r in range(n):
            for R in range(r, n):
                if (L < r < R or L == r < R or r < L < R or r < L == R or r < R < L
                        or L < r == R or L == r == R or r == R < L):
                    out.append((L, r, R))
    return out


def _evaluate(P: _ABCPlan, cut, Q, om, tab, tab_names, la):
    """Batch every heavy factor on the device, then the row-vector chains on the host.
    Chains share prefixes (the same pi row through the same first intervals), so every
    prefix's vector is computed once; every restricted matrix is sliced once."""
    n = Q.shape[0]
    nt = n - 2
    masks = {k: np.isin(np.arange(n), v) for k, v in om.items()}
    masks_t = {k: m[:nt] for k, m in masks.items()}
    tm = [cut[k + 1] - cut[k] for k in range(P.n)][:-1]
    props = la.expm([Q * t for t in tm]) if tm else []
    vl: Dict[Tuple, np.ndarray] = {}
    inf: Dict[Tuple, np.ndarray] = {}
    for key in P.order:
        for ch in P.entries[key][1]:
            for f in ch:
                if f[0] == "VL":
                    vl[(f[1], f[2])] = None
                elif f[0] == "INF":
                    inf[f[1]] = None
    by_k: Dict[int, List[Tuple]] = {}
    for path, k in vl:
        by_k.setdefault(k, []).append(path)
    if by_k and hasattr(la, "vanloan_batch"):
        # every interval's Van Loan paths in one shared evaluation (one job per interval)
        keys = list(masks)
        mid = {kk: i for i, kk in enumerate(keys)}
        mu8 = np.stack([np.asarray(masks[kk], dtype=np.uint8) for kk in keys])
        ks = sorted(by_k)
        job, lens, pm, owner = [], [], [], []
        for j, k in enumerate(ks):
            for path in by_k[k]:
                job.append(j)
                lens.append(len(path))
                pm.extend(mid[w] for w in path)
                owner.append((path, k))
        off = np.zeros(len(job) + 1, dtype=np.int64)
        np.cumsum(lens, out=off[1:])
        t = np.asarray([cut[k + 1] - cut[k] for k in ks], dtype=np.float64)
        res = la.vanloan_batch(Q, mu8, t, np.asarray(job, dtype=np.int32), off,
                               np.asarray(pm, dtype=np.int32)).cpu().numpy()
        for key, m in zip(owner, res):
            vl[key] = m
    else:
        for k, paths in sorted(by_k.items()):
            res = la.vanloan(Q, cut[k + 1] - cut[k], masks, paths)
            for p, m in zip(paths, res):
                vl[(p, k)] = m
    if inf:
        paths = list(inf)
        res = la.deepest(Q[:nt, :nt], masks_t, paths)
        for p, m in zip(paths, res):
            inf[p] = m
    ix = {k: np.asarray(v, dtype=np.int64) for k, v in om.items()}
    name_row = {nm: i for i, nm in enumerate(tab_names)}
    sliced: Dict[Tuple, object] = {}

    def restricted(f):
        m = sliced.get(f)
        if m is None:
            if f[0] == "S":  # identity restricted to (r, c): positions of c inside r
                pos = {s: k for k, s in enumerate(ix[f[1]])}
                m = ("sel", np.asarray([pos[s] for s in ix[f[2]]], dtype=np.int64))
            else:
                M, r, c = ((props[f[1]], f[2], f[3]) if f[0] == "P" else
                           (vl[(f[1], f[2])], f[3], f[4]) if f[0] == "VL" else
                           (inf[f[1]], f[2], f[3]))
                m = ("mat", M[np.ix_(ix[r], ix[c])])
            sliced[f] = m
        return m

    prefix: Dict[Tuple, np.ndarray] = {}
    out = {}
    for key in P.order:
        pn, chains = P.entries[key]
        total = 0.0
        for ch in chains:
            v = tab[name_row[pn]]
            for i in range(len(ch)):
                pk = (pn, ch[:i + 1]) if isinstance(ch, tuple) else (pn, tuple(ch[:i + 1]))
                w = prefix.get(pk)
                if w is None:
                    kind, m = restricted(ch[i])
                    w = v[m] if kind == "sel" else v @ m
                    prefix[pk] = w
                v = w
            total += v.sum()
        out[key] = total
    return out


# ---------------------------------------------------------------------------------------
# emissions (get_emission_prob_mat_introgression, int_get_emission_prob_mat.py:744-1110)
# ---------------------------------------------------------------------------------------


def int_state_specs(t_A, t_B, t_AB, t_C, t_upper, t_out, t_m, coal_AB, coal_BC, coal_ABC,
                    n_int_AB, n_int_ABC, mu_A, mu_B, mu_C, mu_D, mu_AB, mu_ABC, cut_AB,
                    cut_ABC):
    """One spec per hidden state (emissions.state_specs' format), reference order."""
    n = n_int_ABC
    cut_BC = np.concatenate([[0], (np.asarray(cut_AB)[1:] + t_m)])
    specs = []

    def d_vec(jj):
        add = t_upper + cut_ABC[n - 1] - cut_ABC[jj + 1] if jj != n - 1 else 0
        return [t_out, add], [mu_D, mu_ABC]

    def rev(v):
        return list(reversed(v[0])), list(reversed(v[1]))

    def single(a, b, c, ab, first, second, d, state, perm):
        gens = [branch_generator(*a), branch_generator(*rev(b)), branch_generator(*rev(c)),
                branch_generator(*rev(d)), branch_generator(*ab)]
        specs.append((state, 0, perm, gens, first, second, None))

    def double(a, b, c, tt, d, state, perm):
        gens = [branch_generator(*a), branch_generator(*rev(b)), branch_generator(*rev(c)),
                branch_generator(*rev(d)), None]
        specs.append((state, 1, perm, gens, None, None, (tt, mu_ABC)))

    def abc_vecs(i):
        a = ([t_A, t_AB, cut_ABC[i]], [mu_A, mu_AB, mu_ABC])
        b = ([t_B + t_m, t_AB, cut_ABC[i]], [mu_B, mu_AB, mu_ABC])
        c = ([t_C + t_m + t_AB, cut_ABC[i]], [mu_C, mu_ABC])
        return a, b, c

    for i in range(n):
        for j in range(i + 1, n):
            a, b, c = abc_vecs(i)
            ab = ([cut_ABC[j] - cut_ABC[i + 1]], [mu_ABC])
            first = (cut_ABC[i + 1] - cut_ABC[i], mu_ABC, coal_ABC)
            second = ((cut_ABC[j + 1] - cut_ABC[j]) if j != n - 1 else t_upper, mu_ABC,
                      coal_ABC)
            d = d_vec(j)
            single(a, b, c, ab, first, second, d, (1, i, j), 0)
            single(a, c, b, ab, first, second, d, (2, i, j), 1)
            single(b, c, a, ab, first, second, d, (3, i, j), 2)
    for i in range(n):
        a, b, c = abc_vecs(i)
        tt = (cut_ABC[i + 1] - cut_ABC[i]) if i != n - 1 else t_upper
        d = d_vec(i)
        double(a, b, c, tt, d, (1, i, i), 0)
        double(a, c, b, tt, d, (2, i, i), 1)
        double(b, c, a, tt, d, (3, i, i), 2)
    for i in range(n_int_AB):
        for j in range(n):
            a = ([t_A, cut_AB[i]], [mu_A, mu_AB])
            b = ([t_B + t_m, cut_AB[i]], [mu_B, mu_AB])
            c = ([t_C + t_m + t_AB, cut_ABC[j]], [mu_C, mu_ABC])
            ab = ([t_AB - cut_AB[i + 1], cut_ABC[j]], [mu_AB, mu_ABC])
            first = (cut_AB[i + 1] - cut_AB[i], mu_AB, coal_AB)
            second = ((cut_ABC[j + 1] - cut_ABC[j]) if j != n - 1 else t_upper, mu_ABC,
                      coal_ABC)
            single(a, b, c, ab, first, second, d_vec(j), (0, i, j), 0)
    for i in range(n_int_AB):
        for j in range(n):
            a = ([t_B, cut_BC[i]], [mu_B, mu_AB])
            b = ([t_C, cut_BC[i]], [mu_C, mu_AB])
            c = ([t_A, t_AB, cut_ABC[j]], [mu_A, mu_AB, mu_ABC])
            ab = ([t_AB + t_m - cut_BC[i + 1], cut_ABC[j]], [mu_AB, mu_ABC])
            first = (cut_BC[i + 1] - cut_BC[i], mu_AB, coal_BC)
            second = ((cut_ABC[j + 1] - cut_ABC[j]) if j != n - 1 else t_upper, mu_ABC,
                      coal_ABC)
            single(a, b, c, ab, first, second, d_vec(j), (4, i, j), 2)
    return specs


# ---------------------------------------------------------------------------------------
# the entry point
# ---------------------------------------------------------------------------------------


def get_joint_prob_mat_introgression(t_A, t_B, t_AB, t_C, t_m, rho_A, rho_B, rho_AB, rho_C,
                                     rho_ABC, coal_A, coal_B, coal_AB, coal_BC, coal_C,
                                     coal_ABC, m, n_int_AB, n_int_ABC, cut_AB, cut_ABC, la):
    """{(src, dst): probability} of consecutive hidden states
    (int_get_joint_prob_mat.py:16-263)."""
    cut_AB = np.asarray(cut_AB, dtype=float)
    cut_ABC = np.asarray(cut_ABC, dtype=float)
    iv_AB = [cut_AB[i + 1] - cut_AB[i] for i in range(len(cut_AB) - 1)]
    iv_BC = [iv_AB[0] + t_m] + iv_AB[1:]

    sp1 = one_seq(1)
    sym1 = symbols(sp1)
    sp2 = chain_states([1, 2])
    sym2 = symbols(sp2)
    sp3 = chain_states([1, 2, 4])
    sym3 = symbols(sp3)
    sp_miss = MISS_BC
    sym_miss = symbols(sp_miss)

    Q_A = rate_matrix(sym1, coal_A, rho_A)
    Q_B = rate_matrix(sym1, coal_B, rho_B)
    Q_C = rate_matrix(sym1, coal_C, rho_C)
    Q_AB = rate_matrix(sym2, coal_AB, rho_AB)
    Q_BC = rate_matrix(sym2, coal_BC, rho_AB)
    Q_BCm = rate_matrix(sym_miss, coal_BC, rho_AB)
    Q_ABm = rate_matrix(sym_miss, coal_AB, rho_AB)

    # every small exponential of stage 1 in one device batch
    mats = ([Q_A * t_A, Q_B * t_B, Q_C * t_C, Q_A * (t_A + t_AB), Q_C * (t_C + t_m + t_AB),
             Q_B * t_m] + [Q_AB * t for t in iv_AB] + [Q_BC * t for t in iv_BC]
            + [Q_BCm * t for t in iv_BC] + [Q_ABm * t for t in iv_AB])
    E = la.expm(mats)
    final_A, final_B, final_C, final_A_bis, final_C_bis, eB_tm = [e for e in E[:6]]
    final_A, final_B, final_C = final_A[0], final_B[0], final_C[0]
    final_A_bis, final_C_bis = final_A_bis[0], final_C_bis[0]
    k = 6
    nAB = len(iv_AB)
    pr_AB = E[k:k + nAB]
    pr_BC = E[k + nAB:k + 2 * nAB]
    pr_BCm = E[k + 2 * nAB:k + 3 * nAB]
    pr_ABm = E[k + 3 * nAB:k + 4 * nAB]

    sp_B = [_relabel(s, {1: 2}) for s in sp1]
    sp_C = [_relabel(s, {1: 4}) for s in sp1]
    sB_left, fB_left = _split_migration(sp_B, final_B, m, "left")
    sB_right, fB_right = _split_migration(sp_B, final_B, m, "right")

    # right path: migrated B lineages with C (in the AB labels, A standing in for C)
    pi_BC_full = _ordered_start(sp1, sB_right[0:2], final_C, fB_right[0:2], sp2)
    sp_BC = [_relabel(s, {1: 4, 3: 6}) for s in sp2]
    pi_BC_miss = _ordered_start(sp_C, sB_right[2:], final_C, fB_right[2:], sp_miss)
    # left path: B stays, one-sequence chain to the speciation, then with A
    fB_left_full = fB_left[0:2] @ eB_tm
    pi_AB_full = _ordered_start(sp1, sB_left[0:2], final_A, fB_left_full, sp2)
    sp_ABm = [_relabel(s, {4: 1, 6: 3}) for s in sp_miss]
    pi_AB_miss = _ordered_start(sp1, sB_left[2:], final_A, fB_left[2:], sp_ABm)

    chains = {"ABf": _Chain2(sp2, pr_AB, pi_AB_full, 3),
              "ABm": _Chain2(sp_ABm, pr_ABm, pi_AB_miss, 3),
              "BCf": _Chain2(sp_BC, pr_BC, pi_BC_full, 6),
              "BCm": _Chain2(sp_miss, pr_BCm, pi_BC_miss, 6)}
    tab, tab_names = _ab_table(n_int_AB, chains, sp3, final_A_bis, final_C_bis,
                               pi_AB_miss, pi_BC_miss)

    Q3 = rate_matrix(sym3, coal_ABC, rho_ABC)
    om = abc_classes(sp3)
    P = _abc_plan(n_int_AB, tuple(bool(c != np.inf) for c in cut_ABC))
    return _evaluate(P, cut_ABC, Q3, om, tab, tab_names, la)


@lru_cache(maxsize=16)
def _abc_plan(n_int_AB: int, finite: Tuple[bool, ...]) -> "_ABCPlan":
    """The three-sequence table as chains: structural (interval counts and which cutpoints
    are finite), so it is planned once per model size and reused by every evaluation."""
    P = _ABCPlan(np.array([0.0 if f else np.inf for f in finite]))
    _plan_v0_i(P, n_int_AB)
    for L, r, R in _pool_ab_list(P.n):
        _plan_ab_total(P, n_int_AB, L, r, R)
    for l, L, r, R in _pool_abc_list(P.n):
        _plan_abc_pool(P, l, L, r, R)
    return P


def trans_emiss_calc_introgression(t_A, t_B, t_C, t_2, t_upper, t_out, t_m, N_AB, N_BC,
                                   N_ABC, r, m, n_int_AB, n_int_ABC, cut_AB="standard",
                                   cut_ABC="standard", tmp_path="./", la=None):
    """-> (a, b, pi, hidden_names, observed_names), int_get_trans_emiss.py:9-185.  `tmp_path`
    is accepted for the reference's signature (its worker pool pickles shared data there);
    nothing is written."""
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
    t_m = t_m / N_ref
    rho = N_ref * r
    coal_AB = N_ref / N_AB
    coal_BC = N_ref / N_BC
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
    cut_AB = np.asarray(cut_AB, dtype=float)
    cut_ABC = np.asarray(cut_ABC, dtype=float)

    J = get_joint_prob_mat_introgression(
        t_A, t_B, t_AB, t_C, t_m, rho, rho, rho, rho, rho, coal_AB, coal_AB, coal_AB,
        coal_BC, coal_BC, coal_ABC, m, n_int_AB, n_int_ABC, cut_AB, cut_ABC, la)
    hidden = sorted({k[0] for k in J} | {k[1] for k in J})
    expect = 2 * n_int_AB * n_int_ABC + 3 * n_int_ABC + 3 * comb(n_int_ABC, 2, exact=True)
    if len(hidden) != expect:
        raise RuntimeError(f"joint table covers {len(hidden)} states, expected {expect}")
    index = {s: i for i, s in enumerate(hidden)}
    T = np.full((len(hidden), len(hidden)), np.nan)
    for (src, dst), p in J.items():
        T[index[src], index[dst]] = p
    pi = T.sum(axis=1)
    a = T / pi[:, None]

    specs = int_state_specs(t_A, t_B, t_AB, t_C, t_upper, t_out, t_m, coal_AB, coal_BC,
                            coal_ABC, n_int_AB, n_int_ABC, mu, mu, mu, mu, mu, mu, cut_AB,
                            cut_ABC)
    states, rows = emission_rows(specs, la=la)
    pos = {s: i for i, s in enumerate(states)}
    b = rows[[pos[s] for s in hidden]]
    return a, b, pi, dict(enumerate(hidden)), dict(OBSERVED_NAMES)
