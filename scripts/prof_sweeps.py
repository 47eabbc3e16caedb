"""Profiling driver (rocprofv3 target): the chr10 workload of bench.py (BASELINE config 2)
through each sweep entry point separately, so every kernel's counters come from launches of
one configuration: forward (itr_forward_loglik), Viterbi (itr_viterbi), the combined call
(itr_forward_viterbi), posterior at --n-int 7 (post) and 5 (post5).
usage: python scripts/prof_sweeps.py [reps] [fwd,vit,fv,post,post5]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from bench import load_model, make_workload
    from itrails_amd import hmm

    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    which = sys.argv[2].split(",") if len(sys.argv) > 2 else ["fwd", "vit", "fv"]
    a, b, pi, _ = load_model(5)
    W = make_workload("chr10", a, b, pi, 0, 1, 2000.0)
    model, plan = hmm.Model(a, b, pi), hmm.Plan(W["off"])
    d_obs = torch.from_numpy(W["obs"].astype(np.int16)).cuda()
    ll = torch.empty(plan.nblocks, dtype=torch.float64, device="cuda")
    path = torch.empty(plan.total, dtype=torch.uint8, device="cuda")
    post = None
    post5 = None
    if "post5" in which:  # the (5,5) model's posterior over the same 10 Mbp
        plan.reserve(a.shape[0], posterior=True)
        post5 = torch.empty((plan.total, a.shape[0]), dtype=torch.float64, device="cuda")
    if "post" in which:  # config 3: the (7,7) model's posterior over the same 10 Mbp
        a7, b7, pi7, _ = load_model(7)
        W7 = make_workload("chr10", a7, b7, pi7, 0, 1, 2000.0)
        m7, p7 = hmm.Model(a7, b7, pi7), hmm.Plan(W7["off"])
        o7 = torch.from_numpy(W7["obs"].astype(np.int16)).cuda()
        post = torch.empty((p7.total, a7.shape[0]), dtype=torch.float64, device="cuda")
    for _ in range(reps):
        if "post" in which:
            hmm.posterior_device(m7, p7, o7, out=post)
        if "post5" in which:
            hmm.posterior_device(model, plan, d_obs, out=post5)
        if "fwd" in which:
            hmm.forward_loglik_device(model, plan, d_obs, out=ll)
        if "vit" in which:
            hmm.viterbi_device(model, plan, d_obs, out=path)
        if "fv" in which:
            hmm.forward_viterbi_device(model, plan, d_obs, out_ll=ll, out_path=path)
        torch.cuda.synchronize()
    print("done")


if __name__ == "__main__":
    main()
