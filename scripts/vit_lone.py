"""Lone-block Viterbi step latency: one block of T columns ((n,n) KAT model, default (5,5)),
the Viterbi sweep's kernel time / T.  usage: python scripts/vit_lone.py [T] [nblocks] [n_int | i<n_int> (introgression)]"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from itrails_amd import hmm  # noqa: E402
from itrails_amd.synth import sample_alignment  # noqa: E402


def main():
    T = int(sys.argv[1]) if len(sys.argv) > 1 else 18377
    nb = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    arg = sys.argv[3] if len(sys.argv) > 3 else "5"
    if arg.startswith("i"):  # the introgression model, e.g. i5 (N = 95)
        a, b, pi, _ = bench.load_model_intro(int(arg[1:]))
    else:
        a, b, pi, _ = bench.load_model(int(arg))
    obs, off, _ = sample_alignment(a, b, pi, [T] * nb, seed=5)
    model = hmm.Model(a, b, pi)
    plan = hmm.Plan(off)
    plan.reserve(a.shape[0])
    d_obs = torch.from_numpy(obs.astype(np.int16)).cuda()
    d_path = torch.empty(plan.total, dtype=torch.uint8, device="cuda")
    for _ in range(3):
        hmm.viterbi_device(model, plan, d_obs, out=d_path)
    ms = []
    for _ in range(5):
        hmm.viterbi_device(model, plan, d_obs, out=d_path)
        ms.append(hmm.last_kernel_ms("viterbi"))
    m = min(ms)
    print(f"N {a.shape[0]} cfg {os.environ.get('ITR_VIT_CFG', 'default')} T {T} blocks {nb}: viterbi {m:.3f} ms"
          f" = {m * 1e6 / T:.1f} ns/step")


if __name__ == "__main__":
    main()
