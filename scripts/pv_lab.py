"""Prediction-and-verification Viterbi lab: kernel time and (diagnostic library) event counts
and phase cycles on the bench workloads.  usage: python scripts/pv_lab.py [chr10|long|lone]"""
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from itrails_amd import _lib, hmm  # noqa: E402
from itrails_amd.synth import block_lengths, sample_alignment  # noqa: E402

NAMES = {0: "windows", 1: "columns", 2: "mispredicted windows", 3: "scanned pairs",
         4: "gather windows", 8: "cyc predict", 9: "cyc tests+compact", 10: "cyc scans",
         11: "cyc commit", 12: "cyc repair", 13: "cyc between windows"}


def run(kind):
    a, b, pi, _ = bench.load_model(int(os.environ.get("NINT", "5")))
    if kind == "chr10":
        lengths = block_lengths(np.random.default_rng(12345), 10_000_000, 2000.0)
    elif kind == "long":
        lengths = [100_000] * 100
    else:
        lengths = [18377]
    obs, off, _ = sample_alignment(a, b, pi, lengths, seed=777)
    model, plan = hmm.Model(a, b, pi), hmm.Plan(off)
    plan.reserve(a.shape[0])
    d_obs = torch.from_numpy(obs.astype(np.int16)).cuda()
    d_path = torch.empty(plan.total, dtype=torch.uint8, device="cuda")
    ms = []
    for _ in range(4):
        hmm.viterbi_device(model, plan, d_obs, out=d_path)
        ms.append(hmm.last_kernel_ms("viterbi"))
    m = min(ms[1:])
    tot = int(off[-1])
    print(f"{kind}: {len(lengths)} blocks, {tot} columns, longest {max(lengths)}: viterbi "
          f"{m:.3f} ms = {tot / m / 1e3:.1f} M col/s, {m * 1e6 / max(lengths):.1f} ns per "
          f"column of the longest block")
    L = _lib.lib()
    if hasattr(L, "itr_diag_read"):
        buf = (ctypes.c_uint64 * 16)()
        L.itr_diag_read(buf)
        d = list(buf)
        cols = max(d[1], 1)
        for i, name in NAMES.items():
            if d[i]:
                print(f"  {name:22s} {d[i]:14d}  per column {d[i] / cols:9.3f}  per window "
                      f"{d[i] / max(d[0], 1):9.2f}")


if __name__ == "__main__":
    for k in (sys.argv[1:] or ["lone", "long", "chr10"]):
        run(k)
