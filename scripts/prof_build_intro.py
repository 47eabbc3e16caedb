"""cProfile of warm introgression model builds ((n,n), bench.py's INT_KAT parameters).
usage: python scripts/prof_build_intro.py [n_int] [evals]"""
import cProfile
import os
import pstats
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from itrails_amd.optimizer import model_for_introgression  # noqa: E402


def main():
    n_int = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    evals = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    names = list(bench.INT_KAT)
    st = {"n_int_AB": n_int, "n_int_ABC": n_int}

    def ev(i):
        x = [bench.INT_KAT[k] * (1.0 + 1e-3 * ((i + j) % 5 - 2)) for j, k in enumerate(names)]
        return model_for_introgression(x, names, frozenset(["t_1"]), st)

    ev(0)
    for i in range(1, evals + 1):
        t0 = time.perf_counter()
        ev(i)
        print(f"warm build {time.perf_counter() - t0:.3f} s")
    pr = cProfile.Profile()
    pr.enable()
    for i in range(evals):
        ev(100 + i)
    pr.disable()
    s = pstats.Stats(pr)
    s.sort_stats("tottime").print_stats(22)


if __name__ == "__main__":
    main()
