"""Kernel lab: standalone throughput of the forward and Viterbi sweeps on a chosen block-length
distribution (bench.py's synthetic (5,5) columns).  Prints ms per call and CU-ns per column
(= ms x CUs / columns) for itr_forward_loglik, itr_viterbi and itr_forward_viterbi.
usage: python scripts/kernel_lab.py [--mean-block B] [--mbp M] [--reps R] [--which fwd,vit,fv]
Experiment knobs come from the environment of the experiment library (ITR_LIB)."""
import argparse
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mean-block", type=float, default=2000.0)
    ap.add_argument("--mbp", type=float, default=10.0)
    ap.add_argument("--block-len", type=int, default=0)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--which", default="fwd,vit,fv")
    ap.add_argument("--tag", default="")
    ap.add_argument("--check", type=int, default=0)
    args = ap.parse_args()
    import torch
    from bench import load_model, make_workload
    from itrails_amd import hmm

    a, b, pi, _ = load_model(5)
    W = make_workload("chr10", a, b, pi, 0, 1, args.mean_block, args.mbp, args.block_len)
    obs, off = W["obs"], W["off"]
    cols = int(off[-1])
    model, plan = hmm.Model(a, b, pi), hmm.Plan(off)
    plan.reserve(a.shape[0])
    d_obs = torch.from_numpy(obs.astype(np.int16)).cuda()
    ll = torch.empty(plan.nblocks, dtype=torch.float64, device="cuda")
    path = torch.empty(plan.total, dtype=torch.uint8, device="cuda")
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    res = {}
    for w in args.which.split(","):
        f = {"fwd": lambda: hmm.forward_loglik_device(model, plan, d_obs, out=ll),
             "vit": lambda: hmm.viterbi_device(model, plan, d_obs, out=path),
             "fv": lambda: hmm.forward_viterbi_device(model, plan, d_obs, out_ll=ll,
                                                      out_path=path)}[w]
        f()
        torch.cuda.synchronize()
        ts = []
        for _ in range(args.reps):
            t0 = time.perf_counter()
            f()
            torch.cuda.synchronize()
            ts.append((time.perf_counter() - t0) * 1e3)
        ms = float(np.median(ts))
        res[w] = ms
    line = " ".join(f"{w} {ms:.3f} ms ({ms * 1e6 * cus / cols:.1f} CU-ns/col)" for w, ms in res.items())
    print(f"{args.tag} blocks {plan.nblocks} mean {args.mean_block:g} longest {int(np.diff(off).max())}: {line}",
          flush=True)
    if args.check:
        from itrails_amd.tables import build_tables
        from oracle import hmm_oracle as O
        t = build_tables(a, b, pi)
        ref = O.forward_loglik(t, obs, off)
        hmm.forward_loglik_device(model, plan, d_obs, out=ll)
        err_f = np.max(np.abs(ll.cpu().numpy() / ref - 1))
        ref_path = O.viterbi(t, obs, off)
        hmm.viterbi_device(model, plan, d_obs, out=path)
        print(f"{args.tag} check: viterbi paths equal {np.array_equal(path.cpu().numpy(), ref_path)}",
              flush=True)
        hmm.forward_viterbi_device(model, plan, d_obs, out_ll=ll, out_path=path)
        ok_p = np.array_equal(path.cpu().numpy(), ref_path)
        err = np.max(np.abs(ll.cpu().numpy() / ref - 1))
        print(f"{args.tag} check: forward max rel err {err_f:.2e}; combined: paths equal {ok_p}, "
              f"loglik max rel err {err:.2e}", flush=True)


if __name__ == "__main__":
    main()
