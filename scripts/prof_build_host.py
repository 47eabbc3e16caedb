"""Host-side profile of warm (n,n) model builds (config 5's rebuild): cProfile of `evals`
builds, top entries by internal and cumulative time.  usage: python scripts/prof_build_host.py [n_int] [evals]"""
import cProfile
import os
import pstats
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from itrails_amd.optimizer import model_for  # noqa: E402


def main():
    import torch
    n_int = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    evals = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    names = list(bench.KAT)
    st = {"n_int_AB": n_int, "n_int_ABC": n_int}

    def ev(i):
        x = [bench.KAT[k] * (1.0 + 1e-3 * ((i + j) % 5 - 2)) for j, k in enumerate(names)]
        return model_for(x, names, frozenset(["t_1"]), st)

    for i in range(3):
        ev(i)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(evals):
        ev(10 + i)
    torch.cuda.synchronize()
    print(f"warm build {1e3 * (time.perf_counter() - t0) / evals:.3f} ms")
    pr = cProfile.Profile()
    pr.enable()
    for i in range(evals):
        ev(100 + i)
    pr.disable()
    s = pstats.Stats(pr)
    s.sort_stats("tottime").print_stats(40)
    s.sort_stats("cumulative").print_stats(50)


if __name__ == "__main__":
    main()
