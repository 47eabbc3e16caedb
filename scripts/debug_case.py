"""Run one sweep mode on one synthetic case (debugging aid)."""
import sys, os, time
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "tests"))
from test_gpu_sweeps import random_hmm, EDGE_LENGTHS
from itrails_amd import hmm
from itrails_amd.synth import sample_alignment
n = int(sys.argv[1]); mode = sys.argv[2]; which = sys.argv[3]
rng = np.random.default_rng(1000 + n)
a, b, pi = random_hmm(rng, n)
lengths = EDGE_LENGTHS + list(rng.integers(1, 2500, size=40))
if which == "noempty":
    lengths = [L for L in lengths if L > 0]
elif which == "short":
    lengths = [5, 1, 300]
obs, off, _ = sample_alignment(a, b, pi, lengths, seed=n, p_n=0.03, p_gap=0.02)
model, plan = hmm.Model(a, b, pi), hmm.Plan(off)
t0 = time.time()
if mode == "fwd":
    r = hmm.block_logliks(model, plan, obs)
elif mode == "vit":
    r = hmm._paths(model, plan, obs)
else:
    r = hmm._posteriors(model, plan, obs)
print(f"n={n} mode={mode} case={which} ok {time.time()-t0:.3f}s sum={float(np.sum(r))}", flush=True)
