"""Host time of the pieces in front of the Van Loan launch of a warm (5,5) build: the rate
matrix, the job norms, and itr_vanloan_paths' host return (no synchronisation).
usage: python scripts/prof_vl_host.py"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from itrails_amd.optimizer import model_for  # noqa: E402
from itrails_amd.model import linalg as LA  # noqa: E402
from itrails_amd.model.statespace import state_space  # noqa: E402
from itrails_amd import dense  # noqa: E402


def main():
    import torch
    names = list(bench.KAT)
    st = {"n_int_AB": 5, "n_int_ABC": 5}
    cap = {}
    orig = LA.DeviceLinalg.vanloan_batch

    def vb(self, Q, m, t, job, off, pm, job_norm=None):
        cap["a"] = (Q, m, t, job, off, pm)
        return orig(self, Q, m, t, job, off, pm, job_norm)
    LA.DeviceLinalg.vanloan_batch = vb
    for i in range(3):
        x = [bench.KAT[k] * (1.0 + 1e-3 * ((i + j) % 5 - 2)) for j, k in enumerate(names)]
        model_for(x, names, frozenset(["t_1"]), st)
    torch.cuda.synchronize()
    Q, m, t, job, off, pm = cap["a"]
    ss = state_space(3)
    R = 50

    def timeit(label, f):
        f()
        tot = 0.0
        for _ in range(R):  # each call after the device is idle: host time only
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            f()
            tot += time.perf_counter() - t0
        torch.cuda.synchronize()
        print(f"{label:28s} {1e3 * tot / R:7.3f} ms host")
    timeit("rate_matrix(3)", lambda: ss.rate_matrix(1.0, 0.5))
    timeit("vanloan_job_norms", lambda: dense.vanloan_job_norms(Q, t, m, job, off, pm))
    timeit("vanloan_paths (enqueue)", lambda: dense.vanloan_paths(Q, t, m, job, off, pm))
    timeit("torch.empty(out)", lambda: torch.empty((len(job), Q.shape[0], Q.shape[0]),
                                                   dtype=torch.float64, device="cuda"))
    print("paths", len(job), "n", Q.shape[0])


if __name__ == "__main__":
    main()
