"""Per-step latency of the sweep kernels: one long block alone vs many concurrently."""
import os, sys, time, json
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch
from itrails_amd import hmm
from itrails_amd.synth import sample_alignment
g = np.load(os.path.join(ROOT, "tests/golden/model_kat_5_5.npz"))
a, b, pi = g["a"], g["b"], g["pi"]
torch.cuda.set_device(0)
model = hmm.Model(a, b, pi)
out = {}
for label, lengths in [("1x20000", [20000]), ("64x20000", [20000] * 64), ("256x20000", [20000] * 256),
                       ("512x20000", [20000] * 512), ("1024x5000", [5000] * 1024)]:
    obs, off, _ = sample_alignment(a, b, pi, lengths, seed=1)
    plan = hmm.Plan(off)
    d_obs = torch.from_numpy(obs.astype(np.int16)).cuda()
    for _ in range(2):
        hmm.forward_loglik_device(model, plan, d_obs)
        f = hmm.last_kernel_ms("forward")
        hmm.viterbi_device(model, plan, d_obs)
        v = hmm.last_kernel_ms("viterbi")
    T = max(lengths)
    out[label] = {"fwd_ms": f, "vit_ms": v, "fwd_ns_per_step": f * 1e6 / T, "vit_ns_per_step": v * 1e6 / T,
                  "cols_per_s_fwd": off[-1] / f * 1e3, "cols_per_s_vit": off[-1] / v * 1e3}
    print(label, json.dumps(out[label]), flush=True)
