"""Lone-block per-step latency of the forward and Viterbi sweeps (ITR_SWEEP_CFG selects)."""
import os, sys, json
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
T = 20000
obs, off, _ = sample_alignment(a, b, pi, [T], seed=1)
plan = hmm.Plan(off)
d_obs = torch.from_numpy(obs.astype(np.int16)).cuda()
for _ in range(2):
    hmm.forward_loglik_device(model, plan, d_obs)
    f = hmm.last_kernel_ms("forward")
    hmm.viterbi_device(model, plan, d_obs)
    v = hmm.last_kernel_ms("viterbi")
print(os.environ.get("ITR_SWEEP_CFG", "auto"), "fwd ns/step", round(f * 1e6 / T, 1), "vit ns/step", round(v * 1e6 / T, 1), flush=True)
