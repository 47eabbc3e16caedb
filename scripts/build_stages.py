"""Host wall time of the stages of a warm (n,n) model build (trans_emiss_calc): each stage
timed on the host without synchronising (so a stage's time is its host work plus any wait
for the device it contains).  usage: python scripts/build_stages.py [n_int] [evals]"""
import os
import sys
import time
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from itrails_amd.optimizer import model_for  # noqa: E402
from itrails_amd.model import trans_emiss as TE  # noqa: E402
from itrails_amd.model import emissions as EM  # noqa: E402
from itrails_amd.model import chains as CH  # noqa: E402

T = defaultdict(float)


def wrap(mod, name, label):
    f = getattr(mod, name)

    def g(*a, **k):
        t0 = time.perf_counter()
        r = f(*a, **k)
        T[label] += time.perf_counter() - t0
        return r
    setattr(mod, name, g)


def main():
    import torch
    n_int = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    evals = int(sys.argv[2]) if len(sys.argv) > 2 else 30
    for mod, name in ((TE, "prefetch_vanloan"), (TE, "state_specs"), (TE, "emission_rows"),
                      (TE, "joint_prob_mat"), (CH, "run_chain_ab"), (CH, "run_chain_abc"),
                      (TE, "_pair_index"), (EM, "single_table"), (EM, "double_table"),
                      (EM, "generator_matrices")):
        wrap(mod, name, name)
    names = list(bench.KAT)
    st = {"n_int_AB": n_int, "n_int_ABC": n_int}

    def ev(i):
        x = [bench.KAT[k] * (1.0 + 1e-3 * ((i + j) % 5 - 2)) for j, k in enumerate(names)]
        return model_for(x, names, frozenset(["t_1"]), st)

    for i in range(3):
        ev(i)
    torch.cuda.synchronize()
    T.clear()
    t0 = time.perf_counter()
    for i in range(evals):
        ev(10 + i)
    torch.cuda.synchronize()
    tot = (time.perf_counter() - t0) / evals
    print(f"build {1e3 * tot:.3f} ms per evaluation")
    for k, v in sorted(T.items(), key=lambda kv: -kv[1]):
        print(f"  {k:20s} {1e3 * v / evals:7.3f} ms")


if __name__ == "__main__":
    main()
