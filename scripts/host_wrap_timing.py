"""The drop-in wrappers' own stages on the 10 Mbp config-2 layout: Python-side (block
pointers, cached model / plan lookups, the per-block list) and, with ITR_HOST_TIMING=1, the
library's (pack + H2D, sweep, D2H, float64 widening) on stderr.  usage:
ITR_HOST_TIMING=1 python scripts/host_wrap_timing.py [reps]"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from itrails_amd import hmm
    from itrails_amd.synth import block_lengths, sample_alignment
    torch.cuda.init()
    g = np.load(os.path.join(os.path.dirname(__file__), "..", "tests", "golden", "model_kat_5_5.npz"))
    a, b, pi = g["a"], g["b"], g["pi"]
    lengths = block_lengths(np.random.default_rng(12345), 10_000_000, 2000.0)
    obs, off, _ = sample_alignment(a, b, pi, lengths, seed=777)
    V = [obs[off[k]:off[k + 1]].astype(np.int64) for k in range(len(off) - 1)]
    for r in range(int(sys.argv[1]) if len(sys.argv) > 1 else 4):
        T = {}
        t = time.perf_counter()
        lens, ptrs, o2 = hmm._lens_ptrs(V)
        T["lens_ptrs"] = time.perf_counter() - t
        t = time.perf_counter()
        hmm._cached_model(a, b, pi, decode=True)
        T["model_lookup"] = time.perf_counter() - t
        t = time.perf_counter()
        hmm._cached_plan(o2)
        T["plan_lookup"] = time.perf_counter() - t
        t = time.perf_counter()
        hmm.loglik_wrapper(a, b, pi, V)
        T["loglik_wrapper"] = time.perf_counter() - t
        t = time.perf_counter()
        P = hmm.viterbi_wrapper(a, b, pi, V)
        T["viterbi_wrapper"] = time.perf_counter() - t
        t = time.perf_counter()
        x = np.empty(10_000_000)
        x[:] = 1.0
        T["fault_80MB"] = time.perf_counter() - t
        del P, x
        print(" ".join(f"{k} {v * 1e3:.2f}" for k, v in T.items()), flush=True)


if __name__ == "__main__":
    main()
