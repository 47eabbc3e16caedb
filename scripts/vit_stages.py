"""Per-stage cycles of the lone-block Viterbi step (the 9-wave VALU layout, valu_sweep.h
MODE_VIT) from the diagnostic build (libitrails_hip_diag.so: s_memtime stamps around each
stage of every column, one wave per run, ITR_DIAG_WAVE):
  0 publish omega_{t-1} to LDS + staged emission read (+ tile bookkeeping)
  1 the workgroup barrier (waiting for the other waves' publishes)
  2 the max-plus chain (LDS broadcast reads + add / max over the lane's 9 sources)
  3 the three DPP max stages
  4 yd / yo, the stay flag, the new omega
  5 the checkpoint store (first column of a tile)
usage: ITR_LIB=itrails_amd/libitrails_hip_diag.so python scripts/vit_stages.py [T]"""
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from itrails_amd import _lib, hmm  # noqa: E402
from itrails_amd.synth import sample_alignment  # noqa: E402

NAMES = ["publish+ec", "barrier", "chain", "dpp", "final", "ckpt"]


def main():
    T = int(sys.argv[1]) if len(sys.argv) > 1 else 18377
    a, b, pi, _ = bench.load_model(5)
    obs, off, _ = sample_alignment(a, b, pi, [T], seed=5)
    model, plan = hmm.Model(a, b, pi), hmm.Plan(off)
    plan.reserve(a.shape[0])
    d_obs = torch.from_numpy(obs.astype(np.int16)).cuda()
    d_path = torch.empty(plan.total, dtype=torch.uint8, device="cuda")
    L = _lib.lib()
    L.itr_diag_read.argtypes = [ctypes.c_void_p]
    L.itr_diag_read.restype = ctypes.c_int
    for _ in range(2):
        hmm.viterbi_device(model, plan, d_obs, out=d_path)
    torch.cuda.synchronize()
    print(f"T {T}: one block alone, 9-wave layout; cycles per column step (s_memtime)")
    for w in range(9):
        os.environ["ITR_DIAG_WAVE"] = str(w)
        hmm.viterbi_device(model, plan, d_obs, out=d_path)
        ms = hmm.last_kernel_ms("viterbi")
        torch.cuda.synchronize()
        out = np.zeros(16, dtype=np.uint64)
        _lib.check(L.itr_diag_read(out.ctypes.data))
        steps = max(1, int(out[8]))
        per = out[:6].astype(np.float64) / steps
        print(f"wave {w}: " + "  ".join(f"{n} {v:6.1f}" for n, v in zip(NAMES, per)) +
              f"  | sum {per.sum():6.1f} cycles, {ms * 1e6 / T:.1f} ns per column, steps {steps}",
              flush=True)


if __name__ == "__main__":
    main()
