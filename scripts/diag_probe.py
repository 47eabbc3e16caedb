"""Per-segment cycle breakdown of one sweep step (diagnostic build, wave 0 stamps)."""
import ctypes, os, sys, json
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ["ITR_LIB"] = os.path.join(ROOT, "itrails_amd", "libitrails_hip_diag.so")
import torch
from itrails_amd import hmm, _lib
from itrails_amd.synth import sample_alignment
L = _lib.lib()
L.itr_diag_read.argtypes = [ctypes.c_void_p]
g = np.load(os.path.join(ROOT, "tests/golden/model_kat_5_5.npz"))
a, b, pi = g["a"], g["b"], g["pi"]
torch.cuda.set_device(0)
model = hmm.Model(a, b, pi)
names = {"fwd": ["pre-barrier", "barrier", "reads+fma", "combine", "mul", "post"],
         "vit": ["pre-barrier", "barrier", "reads+max", "combine", "tie/M", "post"]}
tag = os.environ.get("ITR_SWEEP_CFG", "auto") + "/" + os.environ.get("ITR_PER_CU", "api") + "/w" + os.environ.get("ITR_DIAG_WAVE", "0")
for label, lengths in [("1x20000", [20000]), ("256x20000", [20000] * 256), ("768x5000", [5000] * 768)]:
    obs, off, _ = sample_alignment(a, b, pi, lengths, seed=1)
    plan = hmm.Plan(off)
    d_obs = torch.from_numpy(obs.astype(np.int16)).cuda()
    for kind in ("fwd", "vit"):
        (hmm.forward_loglik_device if kind == "fwd" else hmm.viterbi_device)(model, plan, d_obs)
        torch.cuda.synchronize()
        ms = hmm.last_kernel_ms("forward" if kind == "fwd" else "viterbi")
        buf = np.zeros(16, dtype=np.uint64)
        _lib.check(L.itr_diag_read(buf.ctypes.data))
        steps = float(buf[8])
        if steps == 0:
            print(tag, label, kind, "no steps recorded by this wave", flush=True)
            continue
        per = {names[kind][i]: round(float(buf[i]) / steps, 1) for i in range(6)}
        tot = sum(per.values())
        T = max(lengths)
        clk = tot * T / (ms * 1e-3) / 1e9  # cycles per step * steps / time
        print(tag, label, kind, json.dumps({"ms": round(ms, 3), "cycles_per_step": round(tot, 1),
              "implied_GHz": round(clk, 3), **per}), flush=True)
