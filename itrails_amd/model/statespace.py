"""Coalescent-with-recombination state spaces of the iTRAILS CTMCs.

A state of the `s`-sequence chain (s = 1, 2, 3 species, two sites each: left and right) is
a set partition of the 2s site-lineages {left_1..left_s, right_1..right_s}: lineages in the
same block have coalesced.  It is written as a restricted-growth label vector of length 2s
(label of every lineage = rank of its block by smallest member), in the enumeration order
of trans_mat.py:51-101 (recursive insertion of the first element into every block of each
partition of the rest, then as a singleton).

Per state:
  * omega = (left, right) bitmasks of the species whose lineage shares its block with
    another lineage of the same site (trans_mat.py:119-209) — 3/5/6 = two species
    coalesced at that site, 7 = all three;
  * transitions (trans_mat.py:212-368): coalescence of two blocks (rate coal) and
    recombination splitting a block that holds both sites' lineages (rate rho), giving
    the rate matrix Q with diagonal -row sum (trans_mat.py:487-508).
"""
from __future__ import annotations

from dataclasses import dataclass
from functools import lru_cache
from itertools import combinations
from typing import Dict, List, Tuple

import numpy as np


def _partitions(items: List[int]):
    """Set partitions in the reference's generation order (trans_mat.py:51-76)."""
    if len(items) == 1:
        yield [[items[0]]]
        return
    head = items[0]
    for rest in _partitions(items[1:]):
        for k in range(len(rest)):
            yield [b if i != k else [head] + b for i, b in enumerate(rest)]
        yield [[head]] + rest


def _canonical(labels) -> Tuple[int, ...]:
    """Relabel to 1..k by increasing value (trans_mat.py:104-117 translate_to_minimum)."""
    order = {v: i + 1 for i, v in enumerate(sorted(set(labels)))}
    return tuple(order[v] for v in labels)


def _omega_bits(labels: Tuple[int, ...], species: int) -> int:
    bits = 0
    for k, v in enumerate(labels):
        if sum(1 for u in labels if u == v) > 1:
            bits += 1 << k
    return bits


@dataclass(frozen=True)
class StateSpace:
    species: int
    states: Tuple[Tuple[int, ...], ...]       # label vectors, index = state number
    index: Dict[Tuple[int, ...], int]          # label vector -> state number
    omega_of: Tuple[Tuple[int, int], ...]      # per state (left, right) omega
    omega_masks: Dict[Tuple[int, int], np.ndarray]   # omega -> bool mask over states
    transitions: Tuple[Tuple[int, int, int], ...]    # (from, to, kind 1=coal / 2=recomb)

    @property
    def n(self) -> int:
        return len(self.states)

    def rate_matrix(self, coal: float, rho: float) -> np.ndarray:
        """Q[from, to] = coal or rho; Q[i, i] = -sum of row i (trans_mat.py:487-508), the row
        sum accumulated left to right like the reference's loop (np.cumsum is sequential).
        The last result is kept (read-only): a build asks for the same matrix twice."""
        last = self.__dict__.get("_rm_last")
        if last is not None and last[0] == (coal, rho):
            return last[1]
        n = self.n
        idx = self.__dict__.get("_tr_idx")
        if idx is None:
            tr = np.asarray(self.transitions, dtype=np.int64).reshape(-1, 3)
            idx = (tr[:, 0], tr[:, 1], tr[:, 2] == 2)
            object.__setattr__(self, "_tr_idx", idx)
        f, t, is_rho = idx
        Q = np.zeros((n, n), dtype=np.float64)
        Q[f, t] = np.where(is_rho, rho, coal)
        d = np.arange(n)
        Q[d, d] = -np.cumsum(Q, axis=1)[:, -1]
        Q.flags.writeable = False
        object.__setattr__(self, "_rm_last", ((coal, rho), Q))
        return Q


@lru_cache(maxsize=None)
def state_space(species: int) -> StateSpace:
    if species not in (1, 2, 3):
        raise ValueError("Species must be 1, 2 or 3")
    m = 2 * species
    states = []
    for part in _partitions(list(range(1, m + 1))):
        lab = [0] * m
        for j, block in enumerate(sorted(part)):
            for v in block:
                lab[v - 1] = j + 1
        states.append(tuple(lab))
    index = {s: i for i, s in enumerate(states)}

    omega_of = []
    masks: Dict[Tuple[int, int], np.ndarray] = {}
    for i, s in enumerate(states):
        om = (_omega_bits(s[:species], species), _omega_bits(s[species:], species))
        omega_of.append(om)
        if om not in masks:
            masks[om] = np.zeros(len(states), dtype=bool)
        masks[om][i] = True

    trans: List[Tuple[int, int, int]] = []
    # coalescence between a left-only and a right-only block, and the reverse recombination
    # (trans_mat.py:212-279)
    for s in states:
        left, right = s[:species], s[species:]
        lset, rset = set(left), set(right)
        if lset == rset:
            continue
        for i in sorted(rset - lset):
            for j in sorted(lset - rset):
                merged = _canonical(left + tuple(j if v == i else v for v in right))
                trans.append((index[s], index[merged], 1))
                trans.append((index[merged], index[s], 2))
    # other coalescences: two blocks meeting at the same site (trans_mat.py:282-368)
    for s in states:
        done = []
        for site in (s[:species], s[species:]):
            if len(set(site)) < 2:
                continue
            for a in range(species):
                for b in range(a + 1, species):
                    x, y = site[a], site[b]
                    if x == y:
                        continue
                    pair = sorted((x, y))
                    if pair in done:
                        continue
                    lo = min(x, y)
                    merged = _canonical(tuple(lo if v in (x, y) else v for v in s))
                    done.append(pair)
                    trans.append((index[s], index[merged], 1))
    return StateSpace(species, tuple(states), index, tuple(omega_of), masks, tuple(trans))


def omega_nonrev_counts(species: int) -> Dict[int, int]:
    """omega bitmask -> number of coalescences it implies (trans_mat.py:511-533)."""
    out = {0: 0}
    mss = [1 << i for i in range(species)]
    for size in range(2, species + 1):
        for sub in combinations(mss, size):
            out[sum(sub)] = size - 1
    return out


# omegas reachable with k coalescences at one site of the 3-sequence chain
# (get_joint_prob_mat.py:164-167)
INVERTED_OMEGA_NONREV_COUNTS_3 = {0: [0], 1: [3, 5, 6], 2: [7]}


def omega_of_key(key) -> Tuple[int, int]:
    """(left, right) omega a path key implies (helper_omegas.py:24-95 translate_to_omega).

    A key side is (kind, first interval, second interval): kind -1 = nothing coalesced yet
    (or both in one interval when the intervals are set), 0 = A,B coalesced in the AB
    epoch, 1/2/3 = the first ABC-epoch coalescence joined (A,B)/(A,C)/(B,C)."""
    def side(k):
        kind, i1, i2 = k
        if kind == -1:
            return 7 if (i1 == i2 and i1 != -1) else 0
        if i2 != -1:
            return 7
        return {0: 3, 1: 3, 2: 5, 3: 6}[kind]
    return side(key[0]), side(key[1])


def masks_without(masks: Dict[Tuple[int, int], np.ndarray], absorbing=(7, 7)):
    """Masks over the non-absorbing states (helper_omegas.py:98-123)."""
    drop = masks[absorbing]
    return {k: v[~drop] for k, v in masks.items() if k != absorbing}
