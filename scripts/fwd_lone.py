"""Lone longest-block forward: one 18,377-column block alone (VALU-only sweep, split halves)
vs the same block among short blocks (hybrid launch: the long block's halves as urgent VALU
tasks on the matrix-core workgroup shape).  usage: python scripts/fwd_lone.py"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from itrails_amd import hmm  # noqa: E402
from itrails_amd.synth import sample_alignment  # noqa: E402


def run(lengths, label):
    a, b, pi, _ = bench.load_model(5)
    obs, off, _ = sample_alignment(a, b, pi, lengths, seed=5)
    model, plan = hmm.Model(a, b, pi), hmm.Plan(off)
    d_obs = torch.from_numpy(obs.astype(np.int16)).cuda()
    out = torch.empty(plan.nblocks, dtype=torch.float64, device="cuda")
    for _ in range(3):
        hmm.forward_loglik_device(model, plan, d_obs, out=out)
    ms = []
    for _ in range(5):
        hmm.forward_loglik_device(model, plan, d_obs, out=out)
        ms.append(hmm.last_kernel_ms("forward"))
    print(f"{label}: forward {min(ms):.3f} ms ({len(lengths)} blocks, {sum(lengths)} columns)")


def main():
    run([18377], "lone 18377 (VALU-only)")
    run([18377] * 100, "100 x 18377 (VALU-only, no groups)")
    run([18377] + [400] * 2000, "18377 + 2000 x 400 (hybrid)")
    run([18377] + [400] * 8000, "18377 + 8000 x 400 (hybrid)")


if __name__ == "__main__":
    main()
