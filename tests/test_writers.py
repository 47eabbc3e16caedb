"""Native result writers (itrails_amd/csrc/writers.cpp) byte-for-byte against the
reference's csv.writer loops (oracle/writers_oracle.py).  CPU only."""
import struct

import numpy as np
import pytest

from itrails_amd import writers as W
from oracle import writers_oracle as O


def test_float_format_matches_python_repr():
    rng = np.random.default_rng(0)
    vals = [0.0, -0.0, 1.0, 0.1, 1e-4, 9.999e-5, 1e-5, 1e16, 9.99e15, 1e15, 123456789012345678.0,
            5e-324, 1.7976931348623157e308, 0.30000000000000004, 2.5, 1e22, 1e-300, 100.0,
            float("inf"), float("-inf"), float("nan")]
    vals += list(rng.random(2000)) + list(rng.random(1000) ** 30) + list(rng.standard_normal(500) * 1e20)
    bits = rng.integers(0, 2**63, size=2000, dtype=np.int64)
    vals += [struct.unpack("d", struct.pack("q", int(b)))[0] for b in bits]
    for v in vals:
        assert W.format_float(v) == repr(float(v)), v


def _paths(rng, nblocks):
    out = []
    for _ in range(nblocks):
        T = int(rng.integers(0, 300))
        runs = np.repeat(rng.integers(0, 70, size=40), rng.integers(1, 30, size=40))[:T]
        out.append(runs.astype(np.float64))
    return out


def _coords(rng, paths):
    out = []
    for p in paths:
        start, strand = int(rng.integers(0, 10**6)), 1 if rng.random() < 0.7 else -1
        c, pos = [], start
        for _ in range(len(p)):
            if rng.random() < 0.1:
                c.append(-9)
            else:
                c.append(pos)
                pos += strand
        if rng.random() < 0.1:
            c = [-9] * len(p)
        out.append(c)
    return out


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_viterbi_csv_bytes(tmp_path, seed):
    rng = np.random.default_rng(seed)
    paths = _paths(rng, 40)
    coords = _coords(rng, paths)
    for cc in (None, coords):
        a, b = tmp_path / "a.csv", tmp_path / "b.csv"
        O.viterbi_csv(a, paths, cc)
        W.write_viterbi_csv(b, paths, cc)
        assert a.read_bytes() == b.read_bytes()


@pytest.mark.parametrize("threads", [1, 3, 16])
def test_posterior_csv_bytes(tmp_path, threads):
    rng = np.random.default_rng(threads)
    post = []
    for _ in range(12):
        T = int(rng.integers(0, 60))
        x = rng.random((T, 7)) ** rng.integers(1, 40, size=(T, 7))
        post.append(x / x.sum(1, keepdims=True) if T else np.zeros((0, 7)))
    coords = _coords(rng, post)
    for cc in (None, coords):
        a, b = tmp_path / "a.csv", tmp_path / "b.csv"
        O.posterior_csv(a, post, cc)
        W.write_posterior_csv(b, post, cc, threads=threads)
        assert a.read_bytes() == b.read_bytes()
    O.posterior_csv(tmp_path / "e1.csv", [])
    W.write_posterior_csv(tmp_path / "e2.csv", [])
    assert (tmp_path / "e1.csv").read_bytes() == (tmp_path / "e2.csv").read_bytes()
