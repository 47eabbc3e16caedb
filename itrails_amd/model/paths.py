"""Omega-path enumeration for the Van Loan and deepest-interval integrals (SURVEY 8a rows
a12, a13, a15).

Within one time interval a site can pass through several omega classes (e.g. nothing
coalesced -> (A,B) coalesced -> all coalesced).  The probability of a given sequence of
classes is a Van Loan integral (vanloan.py:392-425) over the block upper-bidiagonal matrix
built from that sequence; in the last (unbounded) interval it is the deepest-interval
integral (deepest_ti.py:215-256).  These functions enumerate the sequences exactly as the
reference does — depth-first, left site first, then right site, then both — and group them
by the first intermediate class each site passed through ("by" keys), which determines the
topology label of the resulting hidden state.
"""
from __future__ import annotations

from typing import Dict, List, Tuple

Omega = Tuple[int, int]
CODE = {3: 1, 5: 2, 6: 3}  # first two-species coalescence -> topology (deepest_ti.py:179)


def _successors(cur: Omega, start_l: int, start_r: int, end_l: int, end_r: int, nrc, inv,
                by_l: int, by_r: int):
    """(next omega, by_l, by_r) in the reference's visiting order (vanloan.py:107-244)."""
    def tag(by, om, start, end):
        if by != -1:
            return by
        return om if (nrc[om] == 1 and start + 1 != end) else -1
    if start_l < end_l:
        for left in inv[start_l + 1]:
            yield (left, cur[1]), tag(by_l, left, start_l, end_l), by_r
    if start_r < end_r:
        for right in inv[start_r + 1]:
            yield (cur[0], right), by_l, tag(by_r, right, start_r, end_r)
    if start_l < end_l and start_r < end_r:
        for left in inv[start_l + 1]:
            for right in inv[start_r + 1]:
                if nrc[right] > start_r:
                    yield (left, right), tag(by_l, left, start_l, end_l), \
                        tag(by_r, right, start_r, end_r)


def vanloan_paths(omega_init: Omega, omega_fin: Omega, nrc, inv, l_tuple, r_tuple, l_row,
                  r_row, max_num_keys=10, max_per_key=20, max_path_length=15,
                  max_total=200):
    """Sub-paths from omega_init to omega_fin grouped by key (vanloan_identify_wrapper,
    vanloan.py:247-389).  Returns [(key6, [path, ...]), ...] in key discovery order, key6 =
    (topology_l, l_row[1], l_row[2], topology_r, r_row[1], r_row[2]) and each path a tuple of
    omegas starting with omega_init."""
    keys: List[Tuple[int, int]] = []
    groups: Dict[Tuple[int, int], List[Tuple[Omega, ...]]] = {}
    total = [0]
    path: List[Omega] = [tuple(omega_init)]

    def visit(cur: Omega, by_l: int, by_r: int):
        if cur[0] == omega_fin[0] and cur[1] == omega_fin[1]:
            k = (by_l, by_r)
            if k not in groups:
                if len(keys) >= max_num_keys:
                    return
                keys.append(k)
                groups[k] = []
            if len(groups[k]) >= max_per_key or total[0] >= max_total:
                raise RuntimeError("Van Loan path enumeration exceeded the reference's limits")
            groups[k].append(tuple(path))
            total[0] += 1
            return
        sl, sr = nrc[cur[0]], nrc[cur[1]]
        el, er = nrc[omega_fin[0]], nrc[omega_fin[1]]
        for nxt, bl, br in _successors(cur, sl, sr, el, er, nrc, inv, by_l, by_r):
            if len(path) >= max_path_length:
                return
            path.append(nxt)
            visit(nxt, bl, br)
            path.pop()

    visit(tuple(omega_init), -1, -1)
    out = []
    for k in keys:
        tl = 1 if k[0] == 3 else 2 if k[0] == 5 else 3 if k[0] == 6 else l_tuple[0]
        tr = 1 if k[1] == 3 else 2 if k[1] == 5 else 3 if k[1] == 6 else r_tuple[0]
        key6 = (int(tl), int(l_row[1]), int(l_row[2]), int(tr), int(r_row[1]), int(r_row[2]))
        out.append((key6, groups[k]))
    return out


def deepest_paths(omega_init: Omega, absorbing: Omega, nrc, inv, new_path):
    """Sub-paths from omega_init until each site is within one coalescence of the absorbing
    class, grouped by key (deep_identify_wrapper, deepest_ti.py:150-212).  Returns
    [(key6, [path, ...]), ...]."""
    groups: Dict[Tuple[int, int], List[Tuple[Omega, ...]]] = {}
    path: List[Omega] = [tuple(omega_init)]

    def visit(cur: Omega, by_l: int, by_r: int):
        dl = nrc[absorbing[0]] - nrc[cur[0]]
        dr = nrc[absorbing[1]] - nrc[cur[1]]
        if dl <= 1 and dr <= 1:
            groups.setdefault((by_l, by_r), []).append(tuple(path))
            return
        sl, sr = nrc[cur[0]], nrc[cur[1]]
        el, er = nrc[absorbing[0]], nrc[absorbing[1]]
        for nxt, bl, br in _successors(cur, sl, sr, el, er, nrc, inv, by_l, by_r):
            path.append(nxt)
            visit(nxt, bl, br)
            path.pop()

    visit(tuple(omega_init), -1, -1)
    flat = [int(v) for side in new_path for v in side]
    out = []
    for (bl, br), paths in groups.items():
        key6 = list(flat)
        if bl != -1 and key6[0] == -1:
            key6[0] = CODE[bl]
        if br != -1 and key6[3] == -1:
            key6[3] = CODE[br]
        out.append((tuple(key6), paths))
    return out
