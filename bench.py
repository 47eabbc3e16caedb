#!/usr/bin/env python3
"""Benchmark: alignment columns/s for forward + Viterbi on a synthetic 3-species + outgroup
alignment (BASELINE.json config 2: 5 + 5 intervals -> N = 70 hidden states, 10 Mbp per GPU).

One step = the whole decoding hot path over the batch already resident in HBM:
  forward log-likelihood of every MAF block (optimizer.py:145-188) + the log-likelihood
  exchange across ranks (RCCL all-reduce, N > 1) + Viterbi with traceback of every block
  (optimizer.py:305-354).
The HMM is the reference's own (5,5) model build (tests/golden/model_kat_5_5.npz, produced by
trans_emiss_calc with the KAT parameters of SURVEY 8c); columns are sampled from it
(itrails_amd/synth.py), geometric block lengths with mean 2 kbp.

Contract: python bench.py --gpus N --steps K --warmup W ; for N > 1 launched by
torch.distributed.run, one rank per GPU; rank 0 prints ONE JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

FP64_PEAK_TFLOPS = 78.6  # MI355X FP64 (vector = matrix rate), AMD spec


# KAT parameters, internal units of the {t_1} case: times and N times mu,
# r over mu (workflow_optimize.py:360-380)
MU = 2e-8
KAT = {"t_1": 240000.0 * MU, "t_2": 40000.0 * MU, "N_AB": 50000.0 * MU, "N_ABC": 50000.0 * MU,
       "t_upper": 745069.3855 * MU, "r": 1e-8 / MU}


# the introgression model: the KAT set plus B/C admixture 20 kyr before
# the first speciation, {t_1} case (t_B = t_C = t_1 - t_m, int_optimizer.py:504-520),
# admixture proportion m = 0.1 passed as is (the int CLIs would pass m * mu)
INT_KAT = {"t_1": 240000.0 * MU, "t_2": 40000.0 * MU, "N_AB": 50000.0 * MU,
           "N_BC": 40000.0 * MU, "N_ABC": 50000.0 * MU, "t_upper": 745069.3855 * MU,
           "r": 1e-8 / MU, "t_m": 20000.0 * MU, "m": 0.1}


def load_model_intro(n_int: int):
    """The introgression HMM built on the device (model/intro.py) before the timed region."""
    from itrails_amd.config import derive_times_int
    from itrails_amd.model.emissions import cutpoints_ABC
    from itrails_amd.model.intro import trans_emiss_calc_introgression

    d = dict(INT_KAT)
    d = derive_times_int(d, frozenset(["t_1"]), cutpoints_ABC(n_int, 1)[n_int - 1])
    t0 = time.time()
    a, b, pi, _, _ = trans_emiss_calc_introgression(
        d["t_A"], d["t_B"], d["t_C"], d["t_2"], d["t_upper"], d["t_out"], d["t_m"], d["N_AB"],
        d["N_BC"], d["N_ABC"], d["r"], d["m"], n_int, n_int)
    return a, b, pi, (f"itrails introgression ({n_int},{n_int}) model (device-built, "
                      f"{time.time() - t0:.2f} s)")


def load_model(n_int: int):
    f = os.path.join(ROOT, "tests", "golden", f"model_kat_{n_int}_{n_int}.npz")
    if os.path.exists(f):
        g = np.load(f)
        return g["a"], g["b"], g["pi"], f"itrails ({n_int},{n_int}) KAT model"
    # (7,7): the reference build does not finish here; this is the device
    # model build's output for the KAT parameters (scripts/model_timing.py)
    f = os.path.join(ROOT, "tests", "data", f"model_device_{n_int}_{n_int}.npz")
    if os.path.exists(f):
        g = np.load(f)
        return g["a"], g["b"], g["pi"], (f"itrails ({n_int},{n_int}) KAT model, built by the "
                                         "device model build")
    # same state count, random HMM (only until the reference model fixture exists)
    n = {5: 70, 7: 133}.get(n_int, 70)
    g = np.load(os.path.join(ROOT, "tests", "golden", f"sweep_syn{n}.npz"))
    return g["a"], g["b"], g["pi"], f"random N={n} HMM (sweep_syn{n} fixture)"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--n-int", type=int, default=5)
    ap.add_argument("--mode", choices=["fv", "posterior", "optimize"], default="fv",
                    help="fv: forward + Viterbi (BASELINE config 2, the default); posterior: "
                         "posterior decoding (config 3, use --n-int 7); optimize: one "
                         "itrails-optimize objective evaluation per step = device model "
                         "rebuild + forward log-likelihood of the resident columns (config 5)")
    ap.add_argument("--model", choices=["itrails", "introgression"], default="itrails",
                    help="itrails: the plain ILS model (BASELINE configs); introgression: "
                         "the B/C admixture model of itrails-int-* (SURVEY 8(f) row 4), "
                         "built on the device at startup")
    ap.add_argument("--mbp", type=float, default=10.0, help="columns per GPU (Mbp)")
    ap.add_argument("--mean-block", type=float, default=2000.0)
    ap.add_argument("--cpu-sample", type=int, default=10_000_000,
                    help="columns of the bounded CPU-baseline sample (0 = skip)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0,
                    help="repeat the CPU-baseline sample until this much time has passed")
    ap.add_argument("--check", action="store_true", help="verify against the CPU oracle")
    ap.add_argument("--host-path", type=int, default=1,
                    help="1: also time the drop-in wrappers on host NumPy buffers (model "
                         "upload, H2D, sweeps, D2H, float64 paths; reported beside value)")
    ap.add_argument("--concurrent", type=int, default=0,
                    help="1: forward sweep on a side stream beside the Viterbi sweep")
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"],
                    help="collective backend for N > 1 (nccl = RCCL over xGMI; gloo only to "
                         "rehearse the exchange with several ranks on one GPU)")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus and rank == 0:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE {world}", file=sys.stderr)
    local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group("gloo")
    cdev = dev if args.backend == "nccl" else torch.device("cpu")  # collective tensors

    from itrails_amd import hmm
    from itrails_amd.synth import block_lengths, sample_alignment

    intro = args.model == "introgression"
    a, b, pi, model_name = load_model_intro(args.n_int) if intro else load_model(args.n_int)
    n = a.shape[0]
    cols = int(args.mbp * 1e6)
    # identical block-length layout on every rank (weak scaling: the same work per GPU, so
    # the makespan is not set by one rank drawing a longer tail block); content differs
    rng = np.random.default_rng(12345)
    lengths = block_lengths(rng, cols, args.mean_block)
    t0 = time.time()
    obs, off, _ = sample_alignment(a, b, pi, lengths, seed=777 + rank)
    gen_s = time.time() - t0

    model = hmm.Model(a, b, pi)
    plan = hmm.Plan(off)
    post_mode = args.mode == "posterior"
    opt_mode = args.mode == "optimize"
    plan.reserve(n, posterior=post_mode)
    d_obs = torch.from_numpy(obs.astype(np.int16)).to(dev)
    d_ll = torch.empty(plan.nblocks, dtype=torch.float64, device=dev)
    d_path = torch.empty(plan.total, dtype=torch.uint8, device=dev)
    d_post = torch.empty((plan.total, n), dtype=torch.float64, device=dev) if post_mode else None
    nblk_global = plan.nblocks
    if world > 1:
        counts = torch.tensor([plan.nblocks], device=cdev)
        allc = [torch.zeros_like(counts) for _ in range(world)]
        dist.all_gather(allc, counts)
        counts = [int(c.item()) for c in allc]
        nblk_global = sum(counts)
        first = sum(counts[:rank])
        d_ll_global = torch.zeros(nblk_global, dtype=torch.float64, device=cdev)

    fwd_ms, vit_ms, tb_ms = [], [], []
    # forward log-likelihood and Viterbi are independent sweeps over the same resident
    # columns: the forward runs on a side stream beside the Viterbi sweep, so the two
    # kernels share the CUs and the long blocks of one overlap the bulk of the other
    side = torch.cuda.Stream(device=dev) if args.concurrent else None

    build_ms = []
    eval_no = [0]

    def opt_step(timing=False):
        # one objective evaluation at a nearby parameter vector (the simplex moves every
        # call): model rebuild on the device, forward log-likelihood of every block,
        # all-reduce of the per-block values (N > 1), host sum in block order
        from itrails_amd.optimizer import model_for, model_for_introgression

        eval_no[0] += 1
        base = INT_KAT if intro else KAT
        names = list(base)
        x = [base[k] * (1.0 + 1e-3 * ((eval_no[0] + i) % 5 - 2)) for i, k in enumerate(names)]
        tb = time.perf_counter()
        build = model_for_introgression if intro else model_for
        _, (a1, b1, p1, _, _) = build(x, names, frozenset(["t_1"]),
                                      {"n_int_AB": args.n_int, "n_int_ABC": args.n_int})
        m1 = hmm.Model(a1, b1, p1)
        build_ms.append((time.perf_counter() - tb) * 1e3)
        hmm.forward_loglik_device(m1, plan, d_obs, out=d_ll)
        if timing:
            fwd_ms.append(hmm.last_kernel_ms("forward"))
            vit_ms.append(hmm.last_kernel_ms("forward"))
            tb_ms.append(0.0)
        v = d_ll
        if world > 1:
            d_ll_global.zero_()
            d_ll_global[first:first + plan.nblocks] = d_ll.to(cdev)
            dist.all_reduce(d_ll_global)
            v = d_ll_global
        acc = 0.0
        for y in v.cpu().numpy().tolist():
            acc += y
        m1.close()
        return acc

    def step(timing=False):
        if opt_mode:
            opt_step(timing)
            return
        if post_mode:
            hmm.posterior_device(model, plan, d_obs, out=d_post)
            if timing:
                fwd_ms.append(hmm.last_kernel_ms("posterior_fwd"))
                vit_ms.append(hmm.last_kernel_ms("posterior_bwd"))
                tb_ms.append(0.0)
            return
        cur = torch.cuda.current_stream(dev)
        if side is not None and not timing:
            side.wait_stream(cur)
            with torch.cuda.stream(side):
                hmm.forward_loglik_device(model, plan, d_obs, out=d_ll)
            hmm.viterbi_device(model, plan, d_obs, out=d_path)
            cur.wait_stream(side)
        else:
            hmm.forward_loglik_device(model, plan, d_obs, out=d_ll)
        if timing:
            fwd_ms.append(hmm.last_kernel_ms("forward"))
        if world > 1:
            # each rank owns a disjoint slice of the global block vector: the all-reduce is
            # an exact gather (x + 0 = x), and the host sums in block order
            d_ll_global.zero_()
            d_ll_global[first:first + plan.nblocks] = d_ll.to(cdev)
            dist.all_reduce(d_ll_global)
        if side is None or timing:
            hmm.viterbi_device(model, plan, d_obs, out=d_path)
        if timing:
            vit_ms.append(hmm.last_kernel_ms("viterbi"))
            tb_ms.append(hmm.last_kernel_ms("traceback"))

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    if world > 1:
        tt = torch.tensor([dt], dtype=torch.float64, device=cdev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt = float(tt.item())
    # kernel durations (HIP events on the launch stream), separate instrumented passes
    for _ in range(max(1, min(args.steps, 3))):
        step(timing=True)
        torch.cuda.synchronize()

    total_cols = cols * world
    value = total_cols * args.steps / dt
    ll_total = None
    ll_host = (d_ll_global if world > 1 else d_ll).cpu().numpy()
    acc = 0.0
    for v in ll_host.tolist():
        acc += v
    ll_total = acc

    # the drop-in call from host buffers, in a process state like the reference caller's:
    # the resident benchmark buffers (posterior rows, plan workspaces) released first
    host = None
    if args.host_path and not opt_mode and world == 1:
        d_post = None
        plan.close()
        torch.cuda.empty_cache()
        host = host_path_rate(hmm, a, b, pi, obs, off, post_mode)

    result = None
    if rank == 0:
        vit_avg = float(np.mean(vit_ms))
        # Viterbi: one add + one max per (i, j) pair; backward: one FMA
        ops_per_col = 2.0 * n * n
        achieved = ops_per_col * cols / (vit_avg * 1e-3) / 1e12
        traffic, traffic_note = pmc_traffic(n, {"fv": 3, "posterior": 2, "optimize": 0}[args.mode])
        cpu = None
        if opt_mode and intro:
            # the reference's introgression build, timed when its golden model was made in
            # the build container (tests/golden/make_golden.py intmodel; 8 cores shared)
            f = os.path.join(ROOT, "tests", "golden",
                             f"model_int_ikat_{args.n_int}_{args.n_int}.npz")
            if os.path.exists(f):
                sec = float(np.load(f)["build_seconds"])
                cpu = {"value": round(1.0 / sec, 6), "unit": "evaluations/s", "cores": 8,
                       "kind": "reference",
                       "sample": f"trans_emiss_calc_introgression ({args.n_int},{args.n_int}) "
                                 f"{sec:.0f} s in the build container, not re-timed on the "
                                 "GPU box"}
        elif opt_mode:
            # the reference's own model build: 615 s per (5,5) evaluation on the 8-core
            # survey container; it cannot run on the GPU box
            cpu = {"value": round(1.0 / 615.0, 6), "unit": "evaluations/s", "cores": 8,
                   "kind": "reference",
                   "sample": "trans_emiss_calc (5,5) measured once in the build container "
                             "(BASELINE.md 2), not re-timed on the GPU box"}
        elif args.cpu_sample > 0:
            cpu = cpu_baseline(a, b, pi, obs, off, args.cpu_sample, args.cpu_seconds,
                               post_mode)
        check = None
        if args.check and args.mode == "fv":
            check = verify(a, b, pi, obs, off, ll_host if world == 1 else d_ll.cpu().numpy(),
                           d_path.cpu().numpy())
        metric = {"fv": "alignment columns/s (forward+Viterbi), 3sp+outgroup HMM",
                  "posterior": "alignment columns/s (posterior decoding), 3sp+outgroup HMM",
                  "optimize": "itrails-optimize objective evaluations/s (device model rebuild "
                              "+ forward loglik of the resident alignment)"}[args.mode]
        if intro:
            metric = metric.replace("3sp+outgroup HMM", "3sp+outgroup introgression HMM") \
                .replace("itrails-optimize", "itrails-int-optimize")
        if opt_mode:
            value = args.steps / dt
        result = {
            "metric": metric,
            "value": round(value, 4 if opt_mode else 1),
            "unit": "evaluations/s" if opt_mode else "columns/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(dt / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": f"synthetic: columns sampled from the {model_name}, "
                    "geometric blocks mean 2 kbp, 1% gaps + 0.5% N",
            "config": {"workload": f"{args.mbp:g} Mbp/GPU, {n_int_label(args.n_int)}, " +
                                   {"fv": "forward loglik + Viterbi traceback",
                                    "posterior": "posterior decoding",
                                    "optimize": "model rebuild + forward loglik per "
                                                "evaluation"}[args.mode],
                       "hmm": model_name, "hidden_states": n,
                       "columns_per_gpu": cols, "blocks_per_gpu": int(plan.nblocks),
                       "longest_block": int(np.diff(off).max()),
                       "parallelism": f"block-sharded x{world}"},
            "roofline": {"kernel": {"fv": "sweep_kernel<VIT> (Viterbi max-plus)",
                                    "posterior": "sweep_kernel<BWD> (backward + posterior)",
                                    "optimize": "sweep_kernel<FWD_LL> (forward)"}[args.mode],
                         "bound": "mfma",
                         "pipe": ("FP64 VALU (add/max; FP64 vector rate = FP64 matrix rate on "
                                  "MI355X)" if args.mode == "fv" else
                                  "FP64 VALU FMA (FP64 vector rate = FP64 matrix rate on "
                                  "MI355X)"),
                         "achieved": round(achieved, 4), "peak": FP64_PEAK_TFLOPS,
                         "unit": "TFLOP/s", "frac": round(achieved / FP64_PEAK_TFLOPS, 5),
                         # add and max are two VALU instructions per pair (no fused form):
                         # the instruction ceiling is half the FMA-counted FLOP/s figure
                         **({"peak_valu_instr": FP64_PEAK_TFLOPS / 2,
                             "frac_valu_instr": round(achieved / (FP64_PEAK_TFLOPS / 2), 5)}
                            if args.mode == "fv" else {}),
                         "traffic": traffic,
                         "traffic_note": traffic_note,
                         "kernel_ms": round(vit_avg, 4),
                         "forward_ms": round(float(np.mean(fwd_ms)), 4),
                         "traceback_ms": round(float(np.mean(tb_ms)), 4),
                         "algorithmic": f"{ops_per_col:.0f} FP64 ops/column x {cols} columns"},
            "cpu_baseline": cpu,
            **({"build_ms": round(float(np.mean(build_ms)), 1)} if opt_mode else {}),
            **({"host_path": host} if host is not None else {}),
            "loglik_total": ll_total,
            "gen_seconds": round(gen_s, 2),
        }
        if check is not None:
            result["check"] = check
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def host_path_rate(hmm, a, b, pi, obs, off, post_mode, reps=2):
    """The reference-shaped call from host memory: loglik_wrapper + viterbi_wrapper
    (optimizer.py:93, 357) or post_prob_wrapper (241) on a list of NumPy blocks.  Includes
    the model upload, plan creation, the PCIe copies both ways and the float64 path / list
    conversion the reference's callers receive.  Not `value` (inputs resident in HBM)."""
    import torch

    V_lst = [obs[off[k]:off[k + 1]].astype(np.int64) for k in range(len(off) - 1)]
    cols = int(off[-1])
    ts = []
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        if post_mode:
            out = hmm.post_prob_wrapper(a, b, pi, V_lst)
        else:
            hmm.loglik_wrapper(a, b, pi, V_lst)
            out = hmm.viterbi_wrapper(a, b, pi, V_lst)
        ts.append(time.perf_counter() - t0)
        del out
    t = min(ts)
    calls = "post_prob_wrapper" if post_mode else "loglik_wrapper + viterbi_wrapper"
    return {"value": round(cols / t, 1), "unit": "columns/s", "ms": round(t * 1e3, 2),
            "note": f"{calls} on {len(V_lst)} host int64 blocks: model upload, H2D, sweeps, "
                    "D2H and float64 outputs included (best of {reps})".replace("{reps}",
                                                                               str(reps))}


def n_int_label(k):
    return f"{k}+{k} intervals"


def pmc_traffic(n, mode=3):
    """HBM bytes per Viterbi launch from the committed rocprofv3 PMC summary of this same
    command (scripts/gpu_profile.sh -> scripts/summarize_profile.py -> profiles/*_summary.json:
    FETCH_SIZE + WRITE_SIZE, separate passes).  None when no summary for this model size."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_summary.json")))
    for f in reversed(files):
        d = json.load(open(f))
        for name, v in d.items():
            if name.startswith("void itr::sweep_kernel<") and name.endswith(f", {mode}>(itr::SweepArgs)") \
                    and v.get("n_states", 70) == n and "hbm_bytes_raw" in v:
                return round(v["hbm_bytes_raw"]), (
                    f"{os.path.basename(f)} ({name}): FETCH_SIZE+WRITE_SIZE per launch, raw; "
                    "the Viterbi sweep writes the f64 omega rows (padded-state stride) and "
                    "the uint8 stay flags, the posterior sweep the f64 posterior rows")
    return None, "no PMC summary under profiles/"


def cpu_baseline(a, b, pi, obs, off, sample_cols, min_seconds=10.0, posterior=False):
    """The repo's C restatement of the reference sweeps (oracle/, OpenMP over blocks),
    forward + Viterbi on a bounded prefix of this rank's blocks, repeated until min_seconds
    have passed."""
    from itrails_amd.tables import build_tables
    from oracle import hmm_oracle as O

    cores = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or min(os.cpu_count() or 1, 16)
    os.environ["OMP_NUM_THREADS"] = str(cores)
    nb = int(np.searchsorted(off, sample_cols))
    nb = max(1, min(nb, len(off) - 1))
    o2 = off[: nb + 1]
    ob = obs[: o2[-1]]
    t = build_tables(a, b, pi)
    O.lib()
    t0 = time.perf_counter()
    reps = 0
    while True:
        if posterior:
            O.posterior(t, ob, o2)
        else:
            O.forward_loglik(t, ob, o2)
            O.viterbi(t, ob, o2)
        reps += 1
        dt = time.perf_counter() - t0
        if dt >= min_seconds or reps >= 20:
            break
    return {"value": round(float(o2[-1]) * reps / dt, 1), "unit": "columns/s", "cores": cores,
            "kind": "port",
            "sample": f"first {nb} blocks ({int(o2[-1])} columns) of the same workload, "
                      f"{'posterior' if posterior else 'forward + Viterbi'}, {reps} pass(es), "
                      f"{dt:.2f} s"}


def verify(a, b, pi, obs, off, ll, path):
    from itrails_amd.tables import build_tables
    from oracle import hmm_oracle as O

    nb = int(np.searchsorted(off, 300_000))
    o2 = off[: nb + 1]
    t = build_tables(a, b, pi)
    ref_ll = O.forward_loglik(t, obs[: o2[-1]], o2)
    ref_p = O.viterbi(t, obs[: o2[-1]], o2)
    rel = float(np.max(np.abs(ll[:nb] - ref_ll) / np.abs(ref_ll)))
    return {"blocks": nb, "loglik_max_rel_err": rel,
            "viterbi_equal": bool((path[: o2[-1]] == ref_p).all())}


if __name__ == "__main__":
    main()
