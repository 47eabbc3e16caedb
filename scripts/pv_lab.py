"""Lab for the pruned Viterbi (prune_vit.hip) against the 9-wave layout at N = 95 / 133 on the
experiment library (ITR_LIB=itrails_amd/libitrails_hip_exp.so): itr_viterbi's sweep time on
the config-2 layout (mean 2 kbp blocks), on short blocks (mean 300), and on one lone block
(the per-column latency), with the failing-target statistics (ITR_PV_DIAG).
usage: python scripts/pv_lab.py"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from itrails_amd import hmm  # noqa: E402
from itrails_amd.synth import block_lengths, sample_alignment  # noqa: E402


def run(model, off, d_obs, env):
    for k in ("ITR_NO_PRUNE_VIT", "ITR_PV_FORCE", "ITR_PV_DIAG"):
        os.environ.pop(k, None)
    os.environ.update(env)
    plan = hmm.Plan(off)
    plan.reserve(model.n)
    d_path = torch.empty(int(off[-1]), dtype=torch.uint8, device="cuda")
    for _ in range(2):
        hmm.viterbi_device(model, plan, d_obs, out=d_path)
    ms = []
    for _ in range(3):
        hmm.viterbi_device(model, plan, d_obs, out=d_path)
        ms.append(hmm.last_kernel_ms("viterbi"))
    torch.cuda.synchronize()
    os.environ["ITR_PV_DIAG"] = "1"
    hmm.viterbi_device(model, plan, d_obs, out=d_path)
    torch.cuda.synchronize()
    os.environ.pop("ITR_PV_DIAG", None)
    return min(ms), d_path.cpu().numpy()


def main():
    for name, (a, b, pi) in (("(7,7) N=133", bench.load_model(7)[:3]),
                             ("intro (5,5) N=95", bench.load_model_intro(5)[:3])):
        model = hmm.Model(a, b, pi)
        for label, lengths in (("chr10 layout", block_lengths(np.random.default_rng(12345), 10_000_000, 2000.0)),
                               ("short blocks mean 300", block_lengths(np.random.default_rng(1), 3_000_000, 300.0)),
                               ("one block of 18377", np.array([18377]))):
            obs, off, _ = sample_alignment(a, b, pi, lengths, seed=777)
            d_obs = torch.from_numpy(obs.astype(np.int16)).cuda()
            t9, p9 = run(model, off, d_obs, {"ITR_NO_PRUNE_VIT": "1"})
            tp, pp = run(model, off, d_obs, {"ITR_PV_FORCE": "1"})
            cols = int(off[-1])
            print(f"{name} {label}: {len(off) - 1} blocks, {cols} columns, longest {np.diff(off).max()}: "
                  f"9-wave {t9:.3f} ms, pruned {tp:.3f} ms ({tp * 1e6 / np.diff(off).max():.0f} ns per column "
                  f"of the longest), paths equal {np.array_equal(p9, pp)}", flush=True)


if __name__ == "__main__":
    main()
