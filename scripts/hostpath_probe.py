"""Breakdown of the host-buffer posterior path at (7,7), 10 Mbp (bench.py's layout)."""
import time

import numpy as np
import torch

from itrails_amd import hmm
from itrails_amd.synth import block_lengths, sample_alignment
import bench

a, b, pi, _ = bench.load_model(7)
n = a.shape[0]
lengths = block_lengths(np.random.default_rng(12345), 10_000_000, 2000.0)
obs, off, _ = sample_alignment(a, b, pi, lengths, seed=777)
V = [obs[off[k]:off[k + 1]].astype(np.int64) for k in range(len(off) - 1)]
for rep in range(2):
    T = {}
    t = time.perf_counter()
    o, f = hmm.concat_blocks(V); T["pack"] = time.perf_counter() - t
    t = time.perf_counter()
    m, p = hmm.Model(a, b, pi), hmm.Plan(f); T["model+plan"] = time.perf_counter() - t
    t = time.perf_counter()
    out = np.zeros((p.total, n)); T["np.zeros"] = time.perf_counter() - t
    t = time.perf_counter()
    torch.cuda.synchronize()
    from itrails_amd._lib import check, lib, ptr
    check(lib().itr_posterior_host(m.handle, p.handle, ptr(o), ptr(out)))
    T["posterior_host"] = time.perf_counter() - t
    t = time.perf_counter()
    out2 = np.empty((p.total, n)); out2[:] = 1.0; T["fault+fill 10.6GB 1 thread"] = time.perf_counter() - t
    del out, out2
    print(rep, {k: round(v * 1e3, 1) for k, v in T.items()}, flush=True)
for rep in range(2):
    torch.cuda.synchronize()
    t = time.perf_counter()
    res = hmm.post_prob_wrapper(a, b, pi, V)
    print("post_prob_wrapper", round((time.perf_counter() - t) * 1e3, 1), flush=True)
    del res
