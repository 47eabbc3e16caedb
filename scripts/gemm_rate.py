"""Batched FP64 GEMM rate of dense.hip's gemm_kernel (itr_gemm_batched) at model-build shapes."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from itrails_amd.dense import gemm_batched  # noqa: E402

torch.cuda.set_device(0)
for n, batch in ((203, 512), (406, 128), (812, 32), (1015, 16), (2048, 4)):
    A = torch.rand((batch, n, n), dtype=torch.float64, device="cuda")
    B = torch.rand((batch, n, n), dtype=torch.float64, device="cuda")
    gemm_batched(A, B)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    reps = 5
    for _ in range(reps):
        gemm_batched(A, B)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / reps
    print(f"n={n} batch={batch}: {2.0 * n ** 3 * batch / dt / 1e12:.1f} TFLOP/s", flush=True)
