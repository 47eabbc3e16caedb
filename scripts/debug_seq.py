"""Reproduce test_device_layer_matches_host_layer step by step (launch-blocking run)."""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch
from itrails_amd import hmm
torch.cuda.set_device(0)
g = np.load(os.path.join(ROOT, "tests/golden/sweep_syn70.npz"))
off = g["off"]
print("blocks", len(off) - 1, "total", off[-1], "longest", np.diff(off).max(), flush=True)
for frac in ["0", "0.5"]:
    os.environ["ITR_SPLIT_FRAC"] = frac
    model, plan = hmm.Model(g["a"], g["b"], g["pi"]), hmm.Plan(off)
    d_obs = torch.from_numpy(g["obs"].astype(np.int16)).cuda()
    for name, f in [("fwd_dev", lambda: hmm.forward_loglik_device(model, plan, d_obs)),
                    ("host_fwd", lambda: hmm.block_logliks(model, plan, g["obs"])),
                    ("vit_dev", lambda: hmm.viterbi_device(model, plan, d_obs)),
                    ("host_fwd2", lambda: hmm.block_logliks(model, plan, g["obs"])),
                    ("post_dev", lambda: hmm.posterior_device(model, plan, d_obs)),
                    ("host_fwd3", lambda: hmm.block_logliks(model, plan, g["obs"]))]:
        r = f()
        torch.cuda.synchronize()
        print(frac, name, "ok", flush=True)
