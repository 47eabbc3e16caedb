"""Seeded synthetic 3-species + outgroup alignments sampled from an iTRAILS HMM.

The reference ships no example alignment, so benchmarks and large-scale parity
tests draw columns from the HMM itself, vectorised so that 10 Mbp take about a second:

* hidden path per block: the jump chain of `a` with geometric holding times (exactly the
  Markov chain with transition matrix `a`, simulated one sojourn at a time);
* columns: a draw from b[state] (256 N-free symbols, read_data.py:6-15);
* each of the 4 letters is independently replaced by N with probability p_n + p_gap
  (gaps '-' become N in maf_parser, read_data.py:106), giving the ambiguous symbols
  256..624 through the reference alphabet.
Block lengths are geometric with a given mean, seeded.
"""
from __future__ import annotations

import numpy as np

from .read_data import get_obs_state_dct


def _code5_to_index() -> np.ndarray:
    """625-entry table: base-5 code (A,C,T,G,N = 0..4, species 0 most significant) -> symbol."""
    letters = "ACTGN"
    idx = {s: i for i, s in enumerate(get_obs_state_dct())}
    tab = np.zeros(625, dtype=np.uint16)
    for c in range(625):
        s = "".join(letters[(c // 5 ** (3 - k)) % 5] for k in range(4))
        tab[c] = idx[s]
    return tab


def block_lengths(rng, total: int, mean: float, min_len: int = 1) -> np.ndarray:
    """Geometric block lengths (mean `mean`) summing exactly to `total`."""
    out = []
    acc = 0
    while acc < total:
        k = rng.geometric(1.0 / mean, size=max(16, int(2 * (total - acc) / mean) + 16))
        k = np.maximum(k, min_len)
        c = np.cumsum(k)
        take = np.searchsorted(c, total - acc)
        out.append(k[: take + 1])
        acc += int(c[min(take, len(c) - 1)])
    lens = np.concatenate(out).astype(np.int64)
    c = np.cumsum(lens)
    n = int(np.searchsorted(c, total)) + 1
    lens = lens[:n]
    lens[-1] -= int(lens.sum() - total)
    return lens[lens > 0]


def sample_path(rng, a: np.ndarray, pi: np.ndarray, T: int) -> np.ndarray:
    n = a.shape[0]
    stay = np.clip(np.diag(a), 0.0, 1.0 - 1e-15)
    jump = a.copy()
    np.fill_diagonal(jump, 0.0)
    rs = jump.sum(1, keepdims=True)
    jump = np.where(rs > 0, jump / np.where(rs > 0, rs, 1), 1.0 / max(n - 1, 1))
    np.fill_diagonal(jump, 0.0)
    cj = np.cumsum(jump, 1)
    p0 = pi / pi.sum()
    path = np.empty(T, dtype=np.int32)
    s = int(rng.choice(n, p=p0))
    t = 0
    while t < T:
        d = int(rng.geometric(1.0 - stay[s]))
        path[t: t + d] = s
        t += d
        s = int(min(np.searchsorted(cj[s], rng.random() * cj[s, -1], side="right"), n - 1))
    return path


def sample_alignment(a, b, pi, lengths, seed: int = 0, p_n: float = 0.005,
                     p_gap: float = 0.01):
    """Return (obs uint16 [sum(lengths)], off int64 [len+1], hidden path int32)."""
    rng = np.random.default_rng(seed)
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    pi = np.asarray(pi, dtype=np.float64)
    lengths = np.asarray(lengths, dtype=np.int64)
    off = np.zeros(len(lengths) + 1, dtype=np.int64)
    np.cumsum(lengths, out=off[1:])
    total = int(off[-1])
    hidden = np.empty(total, dtype=np.int32)
    for k, T in enumerate(lengths):
        if T:
            hidden[off[k]:off[k + 1]] = sample_path(rng, a, pi, int(T))
    cols = np.empty(total, dtype=np.int64)
    for s in np.unique(hidden):
        sel = np.nonzero(hidden == s)[0]
        p = b[s] / b[s].sum()
        cols[sel] = rng.choice(256, size=len(sel), p=p)
    # base-4 letters (species 0 most significant) -> base-5 with N injection
    digits = np.stack([(cols >> (2 * (3 - k))) & 3 for k in range(4)], axis=1)
    mask = rng.random(digits.shape) < (p_n + p_gap)
    digits = np.where(mask, 4, digits)
    code5 = ((digits[:, 0] * 5 + digits[:, 1]) * 5 + digits[:, 2]) * 5 + digits[:, 3]
    obs = _code5_to_index()[code5]
    return obs.astype(np.uint16), off, hidden


def sample_alignment_range(a, b, pi, lengths, lo: int, hi: int, seed: int = 0,
                           chunk: int = 512, **kw):
    """Blocks [lo, hi) of one large alignment whose content does not depend on how it is
    split: blocks are generated in fixed chunks of `chunk` blocks, chunk c from the seed
    (seed, c), so every rank of a sharded run can sample its own shard and the union over
    ranks is the same alignment for every world size.  Returns (obs, off) of the range,
    off relative to block lo."""
    lengths = np.asarray(lengths, dtype=np.int64)
    if hi <= lo:
        return np.zeros(0, dtype=np.uint16), np.zeros(1, dtype=np.int64)
    parts = []
    for c in range(lo // chunk, (hi - 1) // chunk + 1):
        c0, c1 = c * chunk, min((c + 1) * chunk, len(lengths))
        obs, off, _ = sample_alignment(a, b, pi, lengths[c0:c1], seed=int(seed) * 1_000_003 + c,
                                       **kw)
        s0, s1 = max(lo, c0) - c0, min(hi, c1) - c0
        parts.append(obs[off[s0]:off[s1]])
    off = np.zeros(hi - lo + 1, dtype=np.int64)
    np.cumsum(lengths[lo:hi], out=off[1:])
    return np.concatenate(parts), off


def write_maf(path, obs, off, species, seed: int = 0, p_gap_of_n: float = 0.5,
              chrom_size: int = 250_000_000):
    """Write symbols (obs / off, the 625-letter alphabet of read_data.py:6-24) as a MAF file
    that maf_parser reads back to the same symbols: one alignment block per block, the four
    species in `species` order, every N written as '-' with probability p_gap_of_n (the
    reader maps '-' to N, read_data.py:106), blocks placed one after another on the first
    species' chromosome (+ strand) so parse_coordinates gives positions with -9 at its gaps."""
    rng = np.random.default_rng(seed)
    names = np.array([list(s) for s in get_obs_state_dct()])  # 625 x 4 letters
    pos = 10_000
    with open(path, "w") as f:
        f.write("##maf version=1 scoring=synthetic\n\n")
        for k in range(len(off) - 1):
            cols = names[np.asarray(obs[off[k]:off[k + 1]], dtype=np.int64)]  # T x 4
            if len(cols) == 0:
                continue
            gap = (cols == "N") & (rng.random(cols.shape) < p_gap_of_n)
            cols = np.where(gap, "-", cols)
            f.write("a score=0.0\n")
            for s, name in enumerate(species):
                seq = "".join(cols[:, s])
                size = len(seq) - seq.count("-")
                f.write(f"s {name}.chr1 {pos} {size} + {chrom_size} {seq}\n")
            f.write("\n")
            pos += len(cols) + 100
