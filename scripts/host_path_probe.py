"""Host-path timing of the reference-shaped wrappers on the chr10 workload, call by call:
loglik_wrapper and viterbi_wrapper on 5,036 host int64 blocks.  usage: python scripts/host_path_probe.py"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from itrails_amd import hmm  # noqa: E402
from itrails_amd.synth import block_lengths, sample_alignment  # noqa: E402


def main():
    import torch
    a, b, pi, _ = bench.load_model(5)
    lens = block_lengths(np.random.default_rng(1), 10_000_000, 2000.0)
    obs, off, _ = sample_alignment(a, b, pi, lens, seed=2)
    V = [obs[off[k]:off[k + 1]].astype(np.int64) for k in range(len(off) - 1)]
    for r in range(3):
        for name, f in (("loglik_wrapper", hmm.loglik_wrapper), ("viterbi_wrapper", hmm.viterbi_wrapper)):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            f(a, b, pi, V)
            t1 = time.perf_counter()
            print(f"rep {r} {name:16s} {1e3 * (t1 - t0):8.2f} ms", flush=True)


if __name__ == "__main__":
    main()
