"""Wall time of the device model build (trans_emiss_calc) per interval count, cold and warm,
with a per-phase breakdown from cProfile for the warm call."""
import cProfile, os, pstats, sys, time
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch
from itrails_amd.model.trans_emiss import trans_emiss_calc
torch.cuda.set_device(0)
mu = 2e-8
def args(n):
    t1, t2, tu, N, r = 240000 * mu, 40000 * mu, 745069.3855 * mu, 50000 * mu, 1e-8 / mu
    from itrails_amd.model.emissions import cutpoints_ABC
    c = cutpoints_ABC(n, 1)[n - 1]
    t_out = t1 + t2 + c * N + tu + 2 * N
    return (t1, t1, t1 + t2, t2, tu, t_out, N, N, r, n, n)
for n in [int(x) for x in sys.argv[1:]] or [3, 5]:
    t0 = time.time(); a, b, pi, h, _ = trans_emiss_calc(*args(n)); t1 = time.time()
    pr = cProfile.Profile(); pr.enable()
    a2, b2, pi2, _, _ = trans_emiss_calc(*args(n))
    pr.disable(); t2 = time.time()
    print(f"({n},{n}) N={a.shape[0]} cold {t1 - t0:.2f}s warm {t2 - t1:.2f}s  same={np.array_equal(a, a2)}", flush=True)
    if n == 7:
        np.savez(os.path.join(ROOT, "gpurun_out", f"model_gpu_{n}_{n}.npz"), a=a, b=b, pi=pi)
    st = pstats.Stats(pr); st.sort_stats("cumulative")
    st.print_stats(18)
