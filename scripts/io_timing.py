"""Throughput of the §8(f) host rows: the native MAF reader (csrc/maf.cpp) and the native
result writers (csrc/writers.cpp), each beside the pure-Python restatement of the
reference's code in oracle/ (maf_oracle: the Biopython reader of read_data.py:94-220 as it
behaves; writers_oracle: the csv.writer loops of workflow_viterbi.py:690-743 and
workflow_posterior.py:697-716), on a synthetic 4-species MAF with reference coordinates.

Usage: python scripts/io_timing.py [Mbp] [posterior columns]   (defaults 10, 200000)
"""
import os
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from itrails_amd.maf import maf_parser, parse_coordinates, read_maf  # noqa: E402
from itrails_amd.writers import write_posterior_csv, write_viterbi_csv  # noqa: E402
from oracle import maf_oracle, writers_oracle  # noqa: E402

SP = ["hg38", "panTro5", "gorGor5", "ponAbe2"]


def write_maf(path, total, mean, rng):
    """Blocks of geometric length; gaps and Ns in the sequences, reference gaps included."""
    nt = np.frombuffer(b"ACGTacgtN-", dtype=np.uint8)
    p = np.array([0.2, 0.2, 0.2, 0.2, 0.04, 0.04, 0.04, 0.04, 0.02, 0.02])
    pos, written = 1000, 0
    with open(path, "w") as f:
        f.write("##maf version=1\n\n")
        while written < total:
            T = int(min(total - written, max(1, rng.geometric(1 / mean))))
            f.write("a score=0\n")
            for name in SP:
                seq = nt[rng.choice(10, size=T, p=p)].tobytes().decode()
                f.write(f"s {name}.chr1 {pos} {T} + 100000000 {seq}\n")
            f.write("\n")
            pos += T + 7
            written += T


def timed(fn, *a):
    t0 = time.perf_counter()
    r = fn(*a)
    return r, time.perf_counter() - t0


def main():
    mbp = float(sys.argv[1]) if len(sys.argv) > 1 else 10.0
    npost = int(sys.argv[2]) if len(sys.argv) > 2 else 200_000
    rng = np.random.default_rng(3)
    tmp = tempfile.mkdtemp()
    maf = os.path.join(tmp, "aln.maf")
    write_maf(maf, int(mbp * 1e6), 2000.0, rng)
    mb = os.path.getsize(maf) / 1e6
    print(f"MAF: {mbp:g} Mbp, {mb:.0f} MB", flush=True)

    (obs, off, coords, coff), t = timed(read_maf, maf, SP, "hg38")
    print(f"native read_maf (symbols + coordinates): {t:.2f} s, {mb / t:.0f} MB/s, "
          f"{off[-1] / t / 1e6:.1f} M columns/s", flush=True)
    _, t = timed(maf_parser, maf, SP)
    print(f"native maf_parser (reference types): {t:.2f} s", flush=True)
    _, t2 = timed(parse_coordinates, maf, SP, "hg38")
    print(f"native parse_coordinates (reference types): {t2:.2f} s", flush=True)

    # the pure-Python restatement on a bounded prefix (1/10 of the file)
    small = os.path.join(tmp, "small.maf")
    write_maf(small, int(mbp * 1e5), 2000.0, np.random.default_rng(3))
    smb = os.path.getsize(small) / 1e6
    ref_blocks, t = timed(maf_oracle.maf_parser, small, SP)
    print(f"python restatement maf_parser on {smb:.0f} MB: {t:.2f} s, {smb / t:.1f} MB/s",
          flush=True)
    got = maf_parser(small, SP)
    assert len(got) == len(ref_blocks) and all(np.array_equal(x, y) for x, y in zip(got, ref_blocks))

    # Viterbi segments over all columns (runs of a sticky synthetic path)
    states = np.repeat(rng.integers(0, 70, size=off[-1] // 500 + 1), 500)[: off[-1]].astype(np.uint8)
    out = os.path.join(tmp, "v.csv")
    _, t = timed(write_viterbi_csv, out, states, coords, off)
    print(f"native viterbi.csv with coordinates: {t:.2f} s for {off[-1] / 1e6:.0f} M columns "
          f"({os.path.getsize(out) / 1e6:.1f} MB)", flush=True)
    blocks = [states[off[k]:off[k + 1]].astype(np.float64) for k in range(len(off) - 1)]
    cblocks = [coords[coff[k]:coff[k + 1]].tolist() for k in range(len(coff) - 1)]
    nb = max(1, len(blocks) // 10)
    out2 = os.path.join(tmp, "v2.csv")
    _, t = timed(writers_oracle.viterbi_csv, out2, blocks[:nb], cblocks[:nb])
    cols = sum(len(b) for b in blocks[:nb])
    print(f"python restatement viterbi.csv: {t:.2f} s for {cols / 1e6:.1f} M columns", flush=True)

    # posterior rows (N = 70) for a bounded number of columns
    n = 70
    post = rng.dirichlet(np.ones(n), size=npost)
    poff = np.array([0, npost // 2, npost], dtype=np.int64)
    out3 = os.path.join(tmp, "p.csv")
    _, t = timed(write_posterior_csv, out3, post, None, poff, os.cpu_count() or 1)
    print(f"native posterior.csv: {t:.2f} s for {npost} rows x {n} ({os.path.getsize(out3) / 1e6:.0f} "
          f"MB, {npost / t / 1e6:.2f} M rows/s)", flush=True)
    m = max(1, npost // 20)
    out4 = os.path.join(tmp, "p2.csv")
    _, t = timed(writers_oracle.posterior_csv, out4, [post[:m]])
    print(f"python restatement posterior.csv: {t:.2f} s for {m} rows ({m / t / 1e6:.3f} M rows/s)",
          flush=True)


if __name__ == "__main__":
    main()
