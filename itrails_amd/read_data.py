"""Observed-column alphabet and (later) MAF ingest.

Restates the reference's 4-species column alphabet (read_data.py:6-24) and the expansion
of ambiguous symbols (read_data.py:46-67) with closed-form index arithmetic instead of
list searches, so the 625 x 256 `order` table costs microseconds instead of seconds.

  * symbols 0..255: strings over A,C,T,G for species (A, B, C, outgroup), the first species
    most significant, letter codes A=0, C=1, T=2, G=3;
  * symbols 256..624: the strings over A,C,T,G,N that contain at least one N, in the order of
    the 5-letter enumeration (read_data.py:17-23);
  * order[o]: the N-free symbols an ambiguous symbol stands for, first N outermost, each N
    expanded as A, C, T, G (the recursion of read_data.py:58-67).
"""
from __future__ import annotations

import itertools
from functools import lru_cache

import numpy as np

LETTERS = "ACTG"
NOBS = 625


@lru_cache(maxsize=1)
def get_obs_state_dct() -> list:
    """All 625 observed symbols, in the reference's order (read_data.py:6-24)."""
    names = ["".join(p) for p in itertools.product(LETTERS, repeat=4)]
    names += [
        "".join(p) for p in itertools.product(LETTERS + "N", repeat=4) if "N" in p
    ]
    return names


@lru_cache(maxsize=1)
def _index_of() -> dict:
    return {s: i for i, s in enumerate(get_obs_state_dct())}


def _resolved_index(s: str) -> int:
    v = 0
    for ch in s:
        v = 4 * v + LETTERS.index(ch)
    return v


def get_idx_state(state: int) -> np.ndarray:
    """N-free symbols an observed symbol expands to (read_data.py:46-67)."""
    s = get_obs_state_dct()[state]
    pos = [k for k, ch in enumerate(s) if ch == "N"]
    if not pos:
        return np.array([state], dtype=np.int64)
    out = []
    for fill in itertools.product(LETTERS, repeat=len(pos)):
        chars = list(s)
        for p, ch in zip(pos, fill):
            chars[p] = ch
        out.append(_resolved_index("".join(chars)))
    return np.array(out, dtype=np.int64)


@lru_cache(maxsize=1)
def order_table():
    """The 625 expansions as one CSR table: (flat indices, offsets[626])."""
    order = [get_idx_state(i) for i in range(NOBS)]
    off = np.zeros(NOBS + 1, dtype=np.int64)
    off[1:] = np.cumsum([len(o) for o in order])
    return np.concatenate(order), off


def column_to_index(col: str) -> int:
    """Symbol index of one alignment column string (upper-cased), as maf_parser maps it
    with order_st.index(...) (read_data.py:113-115); raises ValueError like list.index
    for letters outside A/C/T/G/N."""
    try:
        return _index_of()[col.upper()]
    except KeyError:
        raise ValueError(f"{col.upper()!r} is not in list") from None
