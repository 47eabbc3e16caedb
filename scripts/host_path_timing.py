"""Stage times of the drop-in host call (loglik_wrapper + viterbi_wrapper on host NumPy
blocks, BASELINE config 2's 10 Mbp layout): packing, model tables + upload, plan, the
host-buffer sweeps (H2D + sweep + D2H), the float64 path conversion.  usage:
python scripts/host_path_timing.py [reps]"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from itrails_amd import hmm
    from itrails_amd.synth import block_lengths, sample_alignment
    from itrails_amd.tables import build_tables
    torch.cuda.init()
    g = np.load(os.path.join(os.path.dirname(__file__), "..", "tests", "golden", "model_kat_5_5.npz"))
    a, b, pi = g["a"], g["b"], g["pi"]
    lengths = block_lengths(np.random.default_rng(12345), 10_000_000, 2000.0)
    obs, off, _ = sample_alignment(a, b, pi, lengths, seed=777)
    V = [obs[off[k]:off[k + 1]].astype(np.int64) for k in range(len(off) - 1)]
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    for r in range(reps):
        T = {}
        t = time.perf_counter()
        o2, f2 = hmm.concat_blocks(V)
        T["pack"] = time.perf_counter() - t
        t = time.perf_counter()
        tb = build_tables(a, b, pi)
        T["tables"] = time.perf_counter() - t
        t = time.perf_counter()
        m = hmm.Model(tables=tb)
        T["model_create"] = time.perf_counter() - t
        t = time.perf_counter()
        p = hmm.Plan(f2)
        T["plan"] = time.perf_counter() - t
        t = time.perf_counter()
        hmm.block_logliks(m, p, o2)
        T["loglik_host"] = time.perf_counter() - t
        t = time.perf_counter()
        m.prepare_viterbi()
        T["prepare_viterbi"] = time.perf_counter() - t
        t = time.perf_counter()
        path = hmm._paths(m, p, o2)
        T["viterbi_host"] = time.perf_counter() - t
        t = time.perf_counter()
        pf = path.astype(np.float64)
        L = [pf[off[k]:off[k + 1]] for k in range(len(V))]
        T["to_float64_list"] = time.perf_counter() - t
        t = time.perf_counter()
        hmm.loglik_wrapper(a, b, pi, V)
        T["loglik_wrapper"] = time.perf_counter() - t
        t = time.perf_counter()
        hmm.viterbi_wrapper(a, b, pi, V)
        T["viterbi_wrapper"] = time.perf_counter() - t
        T["wrappers_total"] = T["loglik_wrapper"] + T["viterbi_wrapper"]
        print(" ".join(f"{k} {v * 1e3:.2f}" for k, v in T.items()), flush=True)
        m.close()
        p.close()
        del L


if __name__ == "__main__":
    main()
