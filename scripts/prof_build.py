"""Where the time of a warm model build goes: (n,n) KAT build via optimizer.model_for,
wall time per evaluation, then a cProfile of a few warm evaluations (top entries by
cumulative and by internal time).  usage: python scripts/prof_build.py [n_int] [evals]"""
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
    n_int = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    evals = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    names = list(bench.KAT)
    st = {"n_int_AB": n_int, "n_int_ABC": n_int}

    def ev(i):
        x = [bench.KAT[k] * (1.0 + 1e-3 * ((i + j) % 5 - 2)) for j, k in enumerate(names)]
        return model_for(x, names, frozenset(["t_1"]), st)

    t0 = time.perf_counter()
    ev(0)
    print(f"first build {time.perf_counter() - t0:.3f} s")
    ts = []
    for i in range(1, evals + 1):
        t0 = time.perf_counter()
        ev(i)
        ts.append(time.perf_counter() - t0)
    print("warm builds s:", " ".join(f"{t:.3f}" for t in ts))
    # per-call shapes and synchronised times of the batched dense calls
    import torch
    from itrails_amd import dense
    log = []

    def wrap(name, f):
        def g(*a, **k):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            r = f(*a, **k)
            torch.cuda.synchronize()
            x = a[0]
            log.append((name, tuple(x.shape), a[1] if len(a) > 1 and isinstance(a[1], int) else None,
                        time.perf_counter() - t0))
            return r
        return g

    for nm in ("expm_batched", "expm_blocktri_batched", "solve_batched", "gemm_batched"):
        setattr(dense, nm, wrap(nm, getattr(dense, nm)))
    t0 = time.perf_counter()
    ev(50)
    print(f"instrumented build {time.perf_counter() - t0:.3f} s")
    # host-side cost of the Van Loan call (planning + launches, no synchronisation)
    from itrails_amd.model import linalg as LA
    orig = LA.DeviceLinalg.vanloan_batch
    hs = []

    def vb(self, *a, **k):
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        r = orig(self, *a, **k)
        hs.append(time.perf_counter() - t1)
        return r
    LA.DeviceLinalg.vanloan_batch = vb
    for i in range(3):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        ev(60 + i)
        torch.cuda.synchronize()
        print(f"build {time.perf_counter() - t0:.4f} s, vanloan host enqueue {hs[-1] * 1e3:.2f} ms")
    LA.DeviceLinalg.vanloan_batch = orig
    agg = {}
    for name, shp, kb, t in log:
        k = (name, shp, kb)
        c, tt = agg.get(k, (0, 0.0))
        agg[k] = (c + 1, tt + t)
    for k, (c, tt) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        print(f"{k[0]:24s} shape {str(k[1]):20s} kb {k[2]}  calls {c:3d}  total {tt * 1e3:8.2f} ms")
    pr = cProfile.Profile()
    pr.enable()
    for i in range(evals):
        ev(100 + i)
    pr.disable()
    s = pstats.Stats(pr)
    s.sort_stats("cumulative").print_stats(35)
    s.sort_stats("tottime").print_stats(25)


if __name__ == "__main__":
    main()
