#!/usr/bin/env python3
"""Benchmark: alignment columns/s for forward + Viterbi on synthetic 3-species + outgroup
alignments sampled from the iTRAILS (5,5) HMM (N = 70 hidden states), plus the
log-likelihood relative error against the CPU restatement of the reference (BASELINE.json).

Workloads (--workload; default `auto`):
  chr10   BASELINE config 2: one 10 Mbp alignment (5,036 blocks, geometric mean 2 kbp) on one
          GPU — the N = 1 headline.  At N > 1 every rank decodes its own 10 Mbp (weak).
  chr100  BASELINE config 4: ONE fixed 100 Mbp alignment (~50,000 blocks) sharded over the
          ranks with itrails_amd.distributed.shard_ranges (contiguous block ranges balanced by
          columns): strong scaling, the union over ranks is the same alignment at every N.
  auto    chr10 at N = 1, chr100 at N > 1.
One step = the decoding hot path over the rank's columns already resident in HBM: forward
log-likelihood of every block (optimizer.py:145-188), the log-likelihood exchange (one RCCL
all-reduce of the per-block vector, N > 1; optimizer.py:40-65 is the reference's fan-out),
Viterbi with traceback of every block (optimizer.py:305-354).

Contract: python bench.py --gpus N --steps K --warmup W.  For N > 1 either launched by
torch.distributed.run (RANK/WORLD_SIZE/MASTER_* in the environment) or, when WORLD_SIZE is
unset, this script starts its own N rank processes (children, before any GPU call).
Rank 0 prints ONE JSON line.
"""
from __future__ import annotations

import argparse
import glob
import json
import os
import re
import socket
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

FP64_SPEC_TFLOPS = 78.6  # MI355X FP64 vector / matrix (AMD spec, FMA counted as 2 flop)
FP64_SPEC_ADDMAX_TOPS = FP64_SPEC_TFLOPS / 2  # one f64 add or max per lane per issue slot

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


# ---------------------------------------------------------------------------------------
# models
# ---------------------------------------------------------------------------------------
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
        return g["a"], g["b"], g["pi"], f"itrails ({n_int},{n_int}) KAT model (reference build)"
    # no reference output at this size: the device model build's output for the KAT
    # parameters (scripts/model_timing.py)
    f = os.path.join(ROOT, "tests", "data", f"model_device_{n_int}_{n_int}.npz")
    if os.path.exists(f):
        g = np.load(f)
        return g["a"], g["b"], g["pi"], (f"itrails ({n_int},{n_int}) KAT model, built by the "
                                         "device model build")
    raise SystemExit(f"no ({n_int},{n_int}) model fixture")


# ---------------------------------------------------------------------------------------
# workloads
# ---------------------------------------------------------------------------------------
WORKLOADS = {"chr10": 10_000_000, "chr100": 100_000_000}


def make_workload(kind, a, b, pi, rank, world, mean_block, mbp=None, block_len=0):
    """-> dict(obs, off, lo, hi, nblocks, cols_total, cols_local, lengths, scaling).
    block_len > 0: every block that long (the long-block variant), else geometric lengths."""
    from itrails_amd.distributed import shard_ranges
    from itrails_amd.synth import block_lengths, sample_alignment, sample_alignment_range

    cols = int(mbp * 1e6) if mbp else WORKLOADS[kind]
    rng = np.random.default_rng(12345)
    if block_len > 0:
        lengths = np.full(cols // block_len, block_len, dtype=np.int64)
        if cols % block_len:
            lengths = np.append(lengths, cols % block_len)
    else:
        lengths = block_lengths(rng, cols, mean_block)
    if kind == "chr100":
        lo, hi = shard_ranges(lengths, world)[rank]
        obs, off = sample_alignment_range(a, b, pi, lengths, lo, hi, seed=777)
        return dict(obs=obs, off=off, lo=lo, hi=hi, nblocks=len(lengths), cols_total=cols,
                    cols_local=int(off[-1]), lengths=lengths, scaling="strong")
    # chr10: the same block layout on every rank, content per rank (weak scaling at N > 1)
    obs, off, _ = sample_alignment(a, b, pi, lengths, seed=777 + rank)
    nb = len(lengths)
    return dict(obs=obs, off=off, lo=rank * nb, hi=(rank + 1) * nb, nblocks=nb * world,
                cols_total=cols * world, cols_local=cols, lengths=lengths, scaling="weak")


# ---------------------------------------------------------------------------------------
# self-launch of N ranks (when not started by torch.distributed.run)
# ---------------------------------------------------------------------------------------
def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def spawn_ranks(n: int) -> int:
    """Start n child processes of this script, one per GPU, with the torch.distributed
    environment; this process touches no GPU and exits with the worst child status."""
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                   LOCAL_WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:],
                                      env=env))
    rcs = [p.wait() for p in procs]
    return max(rcs, key=abs)


# ---------------------------------------------------------------------------------------
# peaks and counters from profiles/
# ---------------------------------------------------------------------------------------
def valu_peaks():
    """Chip-wide FP64 VALU rates measured by scripts/micro/valu_peak.hip (HIP events), the
    best over 1-8 waves per SIMD: (fma TFLOP/s, add+max Tops/s, source)."""
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "*valu_peak*.txt")))
    if not files:
        return FP64_SPEC_TFLOPS, FP64_SPEC_TFLOPS / 2, "AMD spec (no measured peak)"
    fma, am = 0.0, 0.0
    for line in open(files[-1]):
        m = re.match(r"(\S+)\s+waves/SIMD \d+:\s+\S+ ms\s+(\S+) T", line)
        if m and m.group(1) == "fma":
            fma = max(fma, float(m.group(2)))
        elif m and m.group(1) == "add+max":
            am = max(am, float(m.group(2)))
    return fma, am, os.path.relpath(files[-1], ROOT)


def summary_files():
    """profiles/r*_summary.json, the one recorded for this build of the library first (its
    `library_sha256` entry, written when it was copied in), then by round tag, newest first."""
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_summary.json")), reverse=True)
    h = lib_sha256()

    def this_build(f):
        try:
            return json.load(open(f)).get("library_sha256") == h
        except (OSError, ValueError):
            return False
    return sorted(files, key=lambda f: not this_build(f))  # (stable: tag order kept)


def pmc_traffic(n, mode, tag_hint=""):
    """HBM bytes of the timed call from the committed rocprofv3 PMC summary OF THIS BUILD of
    the library (profiles/r*_summary.json with this library's sha256; scripts/gpu_final.sh ->
    scripts/pmc_summary.py over scripts/prof_sweeps.py: FETCH_SIZE and WRITE_SIZE from
    separate passes, per-dispatch averages).  Summaries of other builds are not used: a
    kernel change makes their bytes stale, and the line then carries null."""
    h = lib_sha256()
    mine = []
    for f in summary_files():
        try:
            if json.load(open(f)).get("library_sha256") == h:
                mine.append(f)
        except (OSError, ValueError):
            pass
    if not mine:
        return None, "no PMC summary of this build of the library under profiles/"

    def fx2(v):
        return v.get("hbm_bytes_fetch_x2", v["hbm_bytes_raw"])

    for f in mine:
        d = json.load(open(f))
        items = [(k, v) for k, v in d.items() if isinstance(v, dict) and
                 v.get("n_states", 70) == n and "hbm_bytes_raw" in v]
        if mode == 3:  # itr_viterbi: every launch of one call
            # the per-wave bulk launch and the reserved sets' late launches (roles 0/1/2, one
            # dispatch each), the long set on both reserved sets (two dispatches), the
            # traceback of the long set
            parts = [(k, v, 2 if "vit_group_kernel<" in k else 1) for k, v in items
                     if "wave_vit_kernel" in k or "vit_group_kernel<" in k or
                     "vit_trace_kernel" in k]
            if any("wave_vit_kernel" in k for k, _, _ in parts):
                return round(sum(fx2(v) * c for _, v, c in parts)), (
                    f"{os.path.basename(f)} (" + " + ".join(
                        (f"2 x " if c == 2 else "") + k for k, _, c in parts) +
                    "): 2 x FETCH_SIZE + WRITE_SIZE per itr_viterbi call, this build "
                    "(gfx950 FETCH correction)")
            continue
        if mode == 2:  # posterior: both launches of the step (forward-store + backward)
            def mode_of(name):
                hm = re.search(r"hybrid_sweep_kernel<\d+, \d+, \d+, (\d+),", name)
                if hm:
                    return int(hm.group(1))
                m = re.search(r"sweep_kernel<[^>]*, (\d+)>\(itr::SweepArgs\)$", name)
                return int(m.group(1)) if m else -1
            parts = [(k, v) for k, v in items if mode_of(k) in (1, 2)]
            if {mode_of(k) for k, _ in parts} == {1, 2}:
                return round(sum(fx2(v) for _, v in parts)), (
                    f"{os.path.basename(f)} (" + " + ".join(k for k, _ in parts) +
                    "): 2 x FETCH_SIZE + WRITE_SIZE per launch, both launches of the step, "
                    "this build (gfx950 FETCH correction)")
            continue
        for name, v in items:
            hyb = re.search(r"hybrid_sweep_kernel<\d+, \d+, \d+, (\d+),", name)
            if (name.startswith("void itr::sweep_kernel<") and
                    name.endswith(f", {mode}>(itr::SweepArgs)")) or \
                    (hyb and int(hyb.group(1)) == mode):
                return round(fx2(v)), (
                    f"{os.path.basename(f)} ({name}): 2 x FETCH_SIZE + WRITE_SIZE per launch, "
                    "this build (gfx950 FETCH correction)")
    return None, "this build's PMC summary holds no launch of this configuration"


def lib_sha256():
    import hashlib
    from itrails_amd import _lib
    return hashlib.sha256(open(_lib.LIB_PATH, "rb").read()).hexdigest()


def fv_call_traffic():
    """HBM bytes per itr_forward_viterbi call (every launch of the call) from the newest
    committed profiles/r*_fv_call_traffic.json (scripts/fv_traffic.py over the FETCH_SIZE /
    WRITE_SIZE passes of the default bench command), only when that profile ran the library
    this run loads (library_sha256): a kernel change makes the old bytes stale, and then the
    line carries null with the old file named."""
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_fv_call_traffic.json")))
    if not files:
        return None, "no per-call PMC traffic under profiles/"
    h = lib_sha256()
    for f in reversed(files):  # the profile of this build, whatever its tag sorts as
        d = json.load(open(f))
        if d.get("library_sha256") == h:
            return d["bytes_per_call"], (
                f"{os.path.basename(f)}: 2 x FETCH_SIZE + WRITE_SIZE of every launch of the "
                f"call ({len(d['per_kernel'])} kernels), this build")
    return None, (f"none of the {len(files)} profiles/r*_fv_call_traffic.json ran this build of "
                  "the library: no traffic for this build")


def pmc_rates(n):
    """Issue and matrix-core counters of the sweep kernels from the latest committed
    rocprofv3 --pmc summary (scripts/gpu_r3g.sh -> scripts/pmc_summary.py): per kernel the
    share of SIMD-cycles with the MFMA pipe busy (SQ_VALU_MFMA_BUSY_CYCLES) and with FP64 VALU
    work issued (SQ_INSTS_VALU x 4 cycles), as shares of all SIMDs of the chip over the
    launch's duration (a launch on a CU subset scores its share of the whole chip), plus the
    waves' waitcnt share (SQ_WAIT_ANY / SQ_WAVE_CYCLES)."""
    for f in summary_files():
        d = json.load(open(f))
        out = {}
        for name, v in d.items():
            if not isinstance(v, dict) or v.get("n_states", 70) != n or "mfma_util" not in v or \
                    not ("sweep_kernel" in name or "wave_" in name):
                continue
            share = 1.0  # shares of all SIMDs of the chip (launches run on CU subsets)
            short = re.sub(r"\(itr::.*$", "", name.replace("void itr::", "")
                           .replace("(anonymous namespace)::", ""))
            out[short] = {"mfma_busy": round(v["mfma_util"] / share, 3),
                          "valu_busy": round(v.get("valu_busy", 0.0) / share, 3),
                          "wait_share": v.get("wait_share")}
        if out:
            return out, os.path.basename(f)
    return None, None


# ---------------------------------------------------------------------------------------
# CPU restatement: checker + baseline (oracle/, test infrastructure; never the product)
# ---------------------------------------------------------------------------------------
def host_threads():
    """Threads of this job's CPU share: OMP_NUM_THREADS when the box sets it (16 per GPU on
    the MI355X pool), else every core."""
    env = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    return env or (os.cpu_count() or 1)


def oracle_check_fv(a, b, pi, obs, off, ll_dev, path_dev, threads):
    """Forward log-likelihood + Viterbi of every block of this rank on the CPU restatement
    (OpenMP over blocks): the relative error of the device log-likelihoods, the path
    equality, and the wall time (the all-cores CPU baseline)."""
    from itrails_amd.tables import build_tables
    from oracle import hmm_oracle as O

    O.set_threads(threads)
    t = build_tables(a, b, pi)
    t0 = time.perf_counter()
    ll_ref = O.forward_loglik(t, obs, off)
    path_ref = O.viterbi(t, obs, off)
    dt = time.perf_counter() - t0
    rel = np.abs(ll_dev - ll_ref) / np.abs(ll_ref)
    acc_d = acc_r = 0.0
    for x, y in zip(ll_dev.tolist(), ll_ref.tolist()):
        acc_d += x
        acc_r += y
    return dict(max_rel=float(rel.max()) if len(rel) else 0.0,
                total_rel=abs(acc_d - acc_r) / abs(acc_r) if acc_r else 0.0,
                equal=bool(np.array_equal(path_dev, path_ref)),
                mismatches=int((path_dev != path_ref).sum()), seconds=dt,
                cols=int(off[-1]))


def oracle_time(a, b, pi, obs, off, sample_cols, threads, posterior):
    """CPU restatement on a bounded prefix: (columns, seconds)."""
    from itrails_amd.tables import build_tables
    from oracle import hmm_oracle as O

    O.set_threads(threads)
    nb = max(1, min(int(np.searchsorted(off, sample_cols)), len(off) - 1))
    o2 = off[: nb + 1]
    ob = obs[: o2[-1]]
    t = build_tables(a, b, pi)
    t0 = time.perf_counter()
    if posterior:
        O.posterior(t, ob, o2)
    else:
        O.forward_loglik(t, ob, o2)
        O.viterbi(t, ob, o2)
    return int(o2[-1]), time.perf_counter() - t0


def oracle_check_post(a, b, pi, obs, off, d_post, threads, chunk_cols=1_000_000):
    """Every posterior row of this rank against the CPU restatement, in runs of whole blocks
    of ~chunk_cols columns (10 Mbp x 133 states is 10.6 GB of rows): allclose at 1e-8, the
    largest relative error over rows > 1e-200, and the restatement's own time (the all-cores
    CPU baseline of posterior mode)."""
    from itrails_amd.tables import build_tables
    from oracle import hmm_oracle as O

    O.set_threads(threads)
    t = build_tables(a, b, pi)
    nb = len(off) - 1
    k0, ok, rel, dt = 0, True, 0.0, 0.0
    while k0 < nb:
        k1 = min(nb, max(k0 + 1, int(np.searchsorted(off, off[k0] + chunk_cols, side="right")) - 1))
        t0 = time.perf_counter()
        ref = O.posterior(t, obs[off[k0]:off[k1]], off[k0:k1 + 1] - off[k0])
        dt += time.perf_counter() - t0
        rows = d_post[int(off[k0]):int(off[k1])].cpu().numpy()
        ok = ok and bool(np.allclose(rows, ref, rtol=1e-8, atol=1e-300))
        big = ref > 1e-200
        if big.any():
            rel = max(rel, float(np.max(np.abs(rows[big] - ref[big]) / ref[big])))
        k0 = k1
    return dict(ok=ok, max_rel=rel, cols=int(off[-1]), seconds=dt)


# ---------------------------------------------------------------------------------------
def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # (defaults: 10 untimed steps bring the GPU to its steady clock first — with 2, the
    # first timed steps ran 2-9 % slower than the calls' own event timers; 20 timed steps)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--workload", choices=["auto", "chr10", "chr100"], default="auto")
    ap.add_argument("--n-int", type=int, default=5)
    ap.add_argument("--mode", choices=["fv", "vit", "posterior", "optimize"], default="fv",
                    help="fv: forward + Viterbi (BASELINE configs 2 and 4, the default); "
                         "vit: Viterbi decoding alone (the itrails-viterbi / viterbi_wrapper "
                         "call); "
                         "posterior: posterior decoding (config 3, use --n-int 7); optimize: "
                         "one itrails-optimize objective evaluation per step = device model "
                         "rebuild + forward log-likelihood of the resident columns (config 5)")
    ap.add_argument("--model", choices=["itrails", "introgression"], default="itrails")
    ap.add_argument("--mbp", type=float, default=None, help="override the workload size")
    ap.add_argument("--mean-block", type=float, default=2000.0)
    ap.add_argument("--block-len", type=int, default=0,
                    help="fixed block length (long-block variant, e.g. 100000: 10 Mbp = 100 "
                         "blocks); 0 = geometric lengths of mean --mean-block")
    ap.add_argument("--verify", type=int, default=1,
                    help="1: check every block against the CPU restatement (log-likelihood "
                         "relative error, Viterbi equality); its timing is the CPU baseline")
    ap.add_argument("--cpu-1core-cols", type=int, default=300_000,
                    help="columns of the 1-core CPU-baseline sample (0 = skip)")
    ap.add_argument("--host-path", type=int, default=1,
                    help="1: also time the drop-in wrappers on host NumPy buffers (N = 1)")
    ap.add_argument("--overlap", type=int, default=1, choices=[0, 1],
                    help="fv mode: 1 = one itr_forward_viterbi call per step (forward sweep "
                         "beside the Viterbi sweep's longest blocks); 0 = the two calls in turn")
    ap.add_argument("--stream", default="side", choices=["side", "default"],
                    help="launch stream of the timed steps: a created stream (side) or the "
                         "legacy default stream, which synchronises implicitly with every "
                         "blocking stream")
    ap.add_argument("--split-build", type=int, default=1, choices=[0, 1],
                    help="optimize mode, N > 1: divide each rebuild's Van Loan work over the "
                         "ranks (one RCCL all-gather) instead of rebuilding on every rank")
    ap.add_argument("--project-shards", type=int, default=0,
                    help="chr100 at N = 1 only: also time each of the W shards a W-GPU run "
                         "would get, alone on this GPU, and report the projected speed-up "
                         "(the N = 1 step / the slowest shard's step)")
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"],
                    help="collective backend for N > 1 (nccl = RCCL over xGMI; gloo only to "
                         "rehearse the exchange with several ranks on one GPU)")
    ap.add_argument("--dist", type=int, default=0, choices=[0, 1],
                    help="1: initialise the process group even at N = 1, so every step's "
                         "log-likelihood exchange is a real collective (RCCL with --backend "
                         "nccl) beside the CU-masked sweep streams")
    args = ap.parse_args()

    if args.gpus > 1 or args.dist:
        # RCCL's own streams beside the launch stream and the three CU-masked streams of
        # itr_forward_viterbi exceed the 4 hardware queues a process gets by default; shared
        # queues serialise.  Set before HIP starts (ranks inherit it).
        os.environ.setdefault("GPU_MAX_HW_QUEUES", "8")
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(args.gpus))

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE {world}")
    local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if args.stream == "side":  # every launch of this process on one created stream
        torch.cuda.set_stream(torch.cuda.Stream(device=dev))
    dist_on = world > 1 or args.dist == 1
    if dist_on:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", str(_free_port()))
        os.environ.setdefault("RANK", "0")
        os.environ.setdefault("WORLD_SIZE", "1")
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group("gloo")
    cdev = dev if args.backend == "nccl" else torch.device("cpu")  # collective tensors
    seen_world = dist.get_world_size() if dist_on else 1

    def allreduce(x, op="sum"):
        if not dist_on:
            return x
        t = torch.tensor([x], dtype=torch.float64, device=cdev)
        dist.all_reduce(t, op={"sum": dist.ReduceOp.SUM, "max": dist.ReduceOp.MAX,
                               "min": dist.ReduceOp.MIN}[op])
        return float(t.item())

    from itrails_amd import hmm

    intro = args.model == "introgression"
    a, b, pi, model_name = load_model_intro(args.n_int) if intro else load_model(args.n_int)
    n = a.shape[0]
    kind = args.workload if args.workload != "auto" else ("chr10" if world == 1 else "chr100")
    t0 = time.time()
    W = make_workload(kind, a, b, pi, rank, world, args.mean_block, args.mbp, args.block_len)
    gen_s = time.time() - t0
    obs, off, lo = W["obs"], W["off"], W["lo"]

    model = hmm.Model(a, b, pi)
    plan = hmm.Plan(off)
    post_mode = args.mode == "posterior"
    opt_mode = args.mode == "optimize"
    vit_mode = args.mode == "vit"
    plan.reserve(n, posterior=post_mode)
    d_obs = torch.from_numpy(obs.astype(np.int16)).to(dev)
    d_ll = torch.empty(plan.nblocks, dtype=torch.float64, device=dev)
    d_path = torch.empty(plan.total, dtype=torch.uint8, device=dev)
    d_post = torch.empty((plan.total, n), dtype=torch.float64, device=dev) if post_mode else None
    d_ll_global = torch.zeros(W["nblocks"], dtype=torch.float64, device=cdev)

    fwd_ms, vit_ms, tb_ms, build_ms, fv_ms = [], [], [], [], []
    eval_no = [0]

    def exchange():
        # each rank owns a disjoint slice of the global block vector: the all-reduce is an
        # exact gather (x + 0 = x); the block-order host sum happens after the timed region
        d_ll_global.zero_()
        d_ll_global[lo:lo + plan.nblocks] = d_ll.to(cdev)
        if dist_on:
            dist.all_reduce(d_ll_global)

    def opt_step(timing=False, xchg=True):
        # one objective evaluation at a nearby parameter vector (the simplex moves every
        # call): model rebuild on the device, forward log-likelihood of every block,
        # all-reduce of the per-block values (N > 1), host sum in block order
        from itrails_amd.optimizer import model_for, model_for_introgression

        eval_no[0] += 1
        base = INT_KAT if intro else KAT
        names = list(base)
        x = [base[k] * (1.0 + 1e-3 * ((eval_no[0] + i) % 5 - 2)) for i, k in enumerate(names)]
        tb = time.perf_counter()
        from itrails_amd.model.linalg import split_build
        build = model_for_introgression if intro else model_for
        with split_build(world > 1 and args.backend == "nccl" and args.split_build == 1):
            _, (a1, b1, p1, _, _) = build(x, names, frozenset(["t_1"]),
                                          {"n_int_AB": args.n_int, "n_int_ABC": args.n_int})
        m1 = hmm.Model(a1, b1, p1)
        if timing:
            build_ms.append((time.perf_counter() - tb) * 1e3)
        hmm.forward_loglik_device(m1, plan, d_obs, out=d_ll)
        if timing:
            fwd_ms.append(hmm.last_kernel_ms("forward"))
        if not xchg:
            m1.close()
            return 0.0
        exchange()
        acc = 0.0
        for y in d_ll_global.cpu().numpy().tolist():
            acc += y
        m1.close()
        return acc

    def step(timing=False, xchg=True):
        if opt_mode:
            opt_step(timing, xchg)
            return
        if post_mode:
            hmm.posterior_device(model, plan, d_obs, out=d_post)
            if timing:
                fwd_ms.append(hmm.last_kernel_ms("posterior_fwd"))
                vit_ms.append(hmm.last_kernel_ms("posterior_bwd"))
            return
        if vit_mode:  # itr_viterbi: sweep + traceback, the path returned to the caller
            hmm.viterbi_device(model, plan, d_obs, out=d_path)
            if timing:
                vit_ms.append(hmm.last_kernel_ms("viterbi"))
                tb_ms.append(hmm.last_kernel_ms("traceback"))
            torch.cuda.current_stream().synchronize()
            return
        if args.overlap and not timing:
            # forward + Viterbi in one call (itr_forward_viterbi): the forward sweep runs
            # beside the Viterbi sweep's longest blocks on a disjoint set of CUs.  A step
            # returns when its outputs are complete, like the reference's wrappers (measured:
            # queueing the next step's fork/join behind the running one costs ~0.7 ms/step)
            hmm.forward_viterbi_device(model, plan, d_obs, out_ll=d_ll, out_path=d_path)
            if xchg:
                exchange()
            torch.cuda.current_stream().synchronize()
            return
        hmm.forward_loglik_device(model, plan, d_obs, out=d_ll)
        if timing:
            fwd_ms.append(hmm.last_kernel_ms("forward"))
        if xchg:
            exchange()
        hmm.viterbi_device(model, plan, d_obs, out=d_path)
        if timing:
            vit_ms.append(hmm.last_kernel_ms("viterbi"))
            tb_ms.append(hmm.last_kernel_ms("traceback"))
            if args.overlap:
                hmm.forward_viterbi_device(model, plan, d_obs, out_ll=d_ll, out_path=d_path)
                fv_ms.append(hmm.last_kernel_ms("forward_viterbi"))

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if dist_on:
        dist.barrier()
    torch.cuda.synchronize()
    # the timed call's own HIP-event duration (fork to join, on its stream), read after every
    # timed step (each fv / vit step ends synchronised, so the read adds no wait): the
    # roofline's kernel_ms comes from the same loop as ms_per_step
    loop_ms = []
    loop_timer = {"fv": "forward_viterbi", "vit": "viterbi"}.get(args.mode) \
        if args.overlap else None
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
        if loop_timer:
            loop_ms.append(hmm.last_kernel_ms(loop_timer))
        if os.environ.get("BENCH_STEP_TIMES"):  # diagnostics only: per-step wall times
            torch.cuda.synchronize()
            print(f"step {(time.perf_counter() - t0) * 1e3:.3f} ms", file=sys.stderr)
    torch.cuda.synchronize()
    if dist_on:
        dist.barrier()
    torch.cuda.synchronize()
    dt = allreduce(time.perf_counter() - t0, "max")
    # kernel durations (HIP events on the launch stream), separate instrumented passes
    for _ in range(max(1, min(args.steps, 3))):
        step(timing=True)
        torch.cuda.synchronize()
    # N > 1: each rank's own step time without the exchange (its share of the work; the
    # timed step waits for the slowest rank inside the all-reduce) and the exchange alone
    per_rank_ms, xchg_ms = None, None
    if dist_on:
        own = []
        for _ in range(max(1, min(args.steps, 3))):
            torch.cuda.synchronize()
            ts = time.perf_counter()
            step(xchg=False)
            torch.cuda.synchronize()
            own.append((time.perf_counter() - ts) * 1e3)
        ex = []
        for _ in range(5):
            dist.barrier()
            torch.cuda.synchronize()
            ts = time.perf_counter()
            exchange()
            torch.cuda.synchronize()
            ex.append((time.perf_counter() - ts) * 1e3)
        mine = torch.tensor([float(np.mean(own)), float(np.median(ex))], dtype=torch.float64,
                            device=cdev)
        allv = [torch.empty_like(mine) for _ in range(world)]
        dist.all_gather(allv, mine)
        per_rank_ms = [round(float(v[0]), 3) for v in allv]
        xchg_ms = round(max(float(v[1]) for v in allv), 4)

    ll_global = d_ll_global.cpu().numpy()
    acc = 0.0
    for v in ll_global.tolist():  # block order, like loglik_wrapper's `acc +=`
        acc += v
    ll_total = acc

    # checks against the CPU restatement, every rank on its own blocks
    threads = host_threads()
    check = None
    if args.verify and args.mode in ("fv", "vit"):
        if vit_mode:  # (the log-likelihoods for the check only)
            hmm.forward_loglik_device(model, plan, d_obs, out=d_ll)
        c = oracle_check_fv(a, b, pi, obs, off, d_ll.cpu().numpy(), d_path.cpu().numpy(), threads)
        check = {"loglik_max_rel_err": allreduce(c["max_rel"], "max"),
                 "loglik_total_rel_err": allreduce(c["total_rel"], "max"),
                 "viterbi_equal": bool(allreduce(1.0 if c["equal"] else 0.0, "min")),
                 "viterbi_mismatched_columns": int(allreduce(c["mismatches"], "sum")),
                 "columns_checked": int(allreduce(c["cols"], "sum")),
                 "reference": "oracle/hmm_oracle.c (CPU restatement of optimizer.py:145-354, "
                              "pinned to the reference's golden vectors)"}
    elif args.verify and post_mode:
        c = oracle_check_post(a, b, pi, obs, off, d_post, threads)
        sums = float((d_post.sum(dim=1) - 1.0).abs().max())
        check = {"posterior_allclose_1e-8": bool(allreduce(1.0 if c["ok"] else 0.0, "min")),
                 "posterior_max_rel_err": allreduce(c["max_rel"], "max"),
                 "columns_checked": int(allreduce(c["cols"], "sum")),
                 "row_sum_max_abs_dev_all_columns": allreduce(sums, "max")}

    # each shard of a W-way split alone on this GPU (chr100, N = 1): the strong-scaling
    # projection of BASELINE config 4 without an 8-GPU node
    shards = None
    if args.project_shards > 1 and kind == "chr100" and world == 1 and args.mode == "fv":
        per = []
        for r in range(args.project_shards):
            Ws = make_workload(kind, a, b, pi, r, args.project_shards, args.mean_block, args.mbp,
                               args.block_len)
            sp = hmm.Plan(Ws["off"])
            sp.reserve(n)
            so = torch.from_numpy(Ws["obs"].astype(np.int16)).to(dev)
            for _ in range(args.warmup):
                hmm.forward_viterbi_device(model, sp, so)
            torch.cuda.synchronize()
            ts = time.perf_counter()
            for _ in range(args.steps):
                hmm.forward_viterbi_device(model, sp, so)
                torch.cuda.current_stream().synchronize()
            per.append(round((time.perf_counter() - ts) / args.steps * 1e3, 4))
            del so
            sp.close()
        step_n1 = dt / args.steps * 1e3
        shards = {"world": args.project_shards, "per_shard_ms": per, "max_ms": max(per),
                  "slowest_rank": int(np.argmax(per)), "n1_step_ms": round(step_n1, 4),
                  "projected_speedup": round(step_n1 / max(per), 3),
                  "note": "each shard's itr_forward_viterbi step alone on this one GPU "
                          "(RCCL all-reduce of the per-block log-likelihoods not included)"}

    # the drop-in call from host buffers (N = 1), resident benchmark buffers released first
    host = None
    if args.host_path and not opt_mode and world == 1:
        d_post = None
        plan.close()
        torch.cuda.empty_cache()
        host = host_path_rate(hmm, a, b, pi, obs, off, post_mode)

    if rank == 0:
        cols_total = W["cols_total"]
        cols_local = W["cols_local"]
        fma_meas, am_meas, peak_src = valu_peaks()
        fma_peak, am_peak = FP64_SPEC_TFLOPS, FP64_SPEC_ADDMAX_TOPS
        fwd_avg = float(np.mean(fwd_ms)) if fwd_ms else 0.0
        vit_avg = float(np.mean(vit_ms)) if vit_ms else 0.0
        tb_avg = float(np.mean(tb_ms)) if tb_ms else 0.0
        pair_ops = 2.0 * n * n  # per column: N^2 FMA (forward / backward) or N^2 add + N^2 max
        step_ms = dt / args.steps * 1e3
        fv_avg = float(np.mean(fv_ms)) if fv_ms else 0.0
        def ideal(fma, am):  # the step's ideal time at the given FP64 rates
            if args.mode == "fv":
                return pair_ops * cols_local / (fma * 1e12) * 1e3 + \
                    pair_ops * cols_local / (am * 1e12) * 1e3
            if vit_mode:
                return pair_ops * cols_local / (am * 1e12) * 1e3
            if post_mode:
                return 2 * pair_ops * cols_local / (fma * 1e12) * 1e3
            return pair_ops * cols_local / (fma * 1e12) * 1e3
        ideal_meas_ms = ideal(fma_meas, am_meas)
        if args.mode == "fv":
            # the timed call itself (itr_forward_viterbi, fork to join): its ideal time at
            # the FP64 spec rates, forward at the FMA rate and Viterbi at the add+max rate
            ideal_ms = ideal(fma_peak, am_peak)
            dom = ("itr_forward_viterbi: hybrid_sweep_kernel<FWD_LL> (forward VALU halves, "
                   "reserved CUs) | vit_group_kernel (longest blocks' Viterbi, reserved CUs) | "
                   "wave_mixed_kernel (forward groups + per-wave Viterbi, the rest)")
            dom_ms = float(np.mean(loop_ms)) if loop_ms else (fv_avg if fv_avg else vit_avg)
            dom_peak = 2 * pair_ops * cols_local / (ideal_ms * 1e-3) / 1e12  # combined peak
            dom_mode = 3
        elif vit_mode:
            dom, dom_ms, dom_peak, dom_mode = ("Viterbi max-plus sweep: vit_group_kernel (longest "
                                               "blocks, both reserved CU sets) | wave_vit_kernel "
                                               "(rest)"), \
                float(np.mean(loop_ms)) if loop_ms else vit_avg, am_peak, 3
            ideal_ms = ideal(fma_peak, am_peak)
        elif post_mode:
            # the whole itr_posterior step (forward-store launch + backward launch, 4 N^2
            # flop per column) against the FMA peak
            hyb = 65 <= n <= 72 or 129 <= n <= 144  # (mfma_sweeps.hip kMCfgs: post = true)
            dom = ("itr_posterior: hybrid_sweep_kernel<FWD_STORE> + hybrid_sweep_kernel<BWD> "
                   "(matrix-core groups + VALU tasks of the longest blocks)") if hyb else \
                ("itr_posterior: sweep_kernel<FWD_STORE> + sweep_kernel<BWD> (VALU)")
            dom_ms, dom_peak, dom_mode = step_ms, fma_peak, 2
            ideal_ms = ideal(fma_peak, am_peak)
        else:
            dom, dom_ms, dom_peak, dom_mode = "sweep_kernel<FWD_LL> (forward)", fwd_avg, \
                fma_peak, 0
            ideal_ms = ideal(fma_peak, am_peak)
        dom_ops = (2 if args.mode in ("fv", "posterior") else 1) * pair_ops * cols_local
        achieved = dom_ops / (dom_ms * 1e-3) / 1e12 if dom_ms else 0.0
        # the profiled workloads: the chr10 layout at N = 70 (every entry point) and N = 133
        # (posterior) — scripts/prof_sweeps.py; other layouts carry no traffic
        profiled = kind == "chr10" and not intro and args.block_len == 0 and args.mbp is None
        default_fv = args.mode == "fv" and n == 70 and profiled
        if default_fv:
            traffic, traffic_note = fv_call_traffic()
        elif profiled and args.mode != "fv":
            traffic, traffic_note = pmc_traffic(n, dom_mode)
        else:
            traffic, traffic_note = None, "no PMC profile of this workload under profiles/"
        rates, rates_src = pmc_rates(n)
        cpu = None
        if opt_mode:
            f = os.path.join(ROOT, "tests", "golden",
                             f"model_int_ikat_{args.n_int}_{args.n_int}.npz" if intro else
                             f"model_kat_{args.n_int}_{args.n_int}.npz")
            if os.path.exists(f) and "build_seconds" in np.load(f):
                sec = float(np.load(f)["build_seconds"])
                cpu = {"value": round(1.0 / sec, 6), "unit": "evaluations/s", "cores": 8,
                       "kind": "reference",
                       "sample": f"the reference's model build ({args.n_int},{args.n_int}) took "
                                 f"{sec:.0f} s in the 8-core build container "
                                 "(tests/golden/make_golden.py), not re-timed on the GPU box"}
        elif world == 1:
            # all cores of this job's share: the verification pass over the whole workload
            # (fv) or the posterior check sample; 1 core: a bounded prefix
            if check is not None:
                ccols, csec = c["cols"], c["seconds"]
            else:
                ccols, csec = oracle_time(a, b, pi, obs, off, 2_000_000, threads, post_mode)
            one = None
            if args.cpu_1core_cols > 0:
                c1, s1 = oracle_time(a, b, pi, obs, off, args.cpu_1core_cols, 1, post_mode)
                one = {"value": round(c1 / s1, 1), "cores": 1,
                       "sample": f"first {c1} columns, {s1:.2f} s"}
            cpu = {"value": round(ccols / csec, 1), "unit": "columns/s", "cores": threads,
                   "host_cpu_count": os.cpu_count(), "kind": "port",
                   "sample": f"{'posterior' if post_mode else 'forward + Viterbi'} over "
                             f"{ccols} columns of this workload, {csec:.2f} s on {threads} "
                             "threads (OMP_NUM_THREADS = this job's CPU share)",
                   "one_core": one}
        metric = {"fv": "alignment columns/s (forward+Viterbi), 3sp+outgroup HMM",
                  "vit": "alignment columns/s (Viterbi decoding), 3sp+outgroup HMM",
                  "posterior": "alignment columns/s (posterior decoding), 3sp+outgroup HMM",
                  "optimize": "itrails-optimize objective evaluations/s (device model rebuild "
                              "+ forward loglik of the resident alignment)"}[args.mode]
        if intro:
            metric = metric.replace("3sp+outgroup HMM", "3sp+outgroup introgression HMM") \
                .replace("itrails-optimize", "itrails-int-optimize")
        value = args.steps / dt if opt_mode else cols_total * args.steps / dt
        result = {
            "metric": metric,
            "value": round(value, 4 if opt_mode else 1),
            "unit": "evaluations/s" if opt_mode else "columns/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(step_ms, 4),
            "higher_is_better": True,
            "scaling": W["scaling"],
            "vs_baseline": None,
            "dtype": "f64",
            "data": f"synthetic: columns sampled from the {model_name}, " +
                    (f"blocks of {args.block_len} columns" if args.block_len > 0 else
                     f"geometric blocks mean {args.mean_block:g} columns") +
                    ", 1% gaps + 0.5% N",
            "config": {"workload": f"{kind}: {cols_total / 1e6:g} Mbp " +
                                   ("alignment sharded over the ranks" if W["scaling"] == "strong"
                                    else "per GPU") + f", {args.n_int}+{args.n_int} intervals, " +
                                   {"fv": "forward loglik + Viterbi traceback",
                                    "vit": "Viterbi sweep + traceback",
                                    "posterior": "posterior decoding",
                                    "optimize": "model rebuild + forward loglik per "
                                                "evaluation"}[args.mode],
                       "hmm": model_name, "hidden_states": n,
                       "columns_total": cols_total, "blocks_total": int(W["nblocks"]),
                       "columns_rank0": cols_local, "blocks_rank0": int(plan.nblocks),
                       "longest_block_rank0": int(np.diff(off).max()) if plan.nblocks else 0,
                       "parallelism": f"block-sharded x{world}",
                       "world_size_seen": seen_world,
                       "backend": (dist.get_backend() if dist_on else None)},
            "roofline": {"kernel": dom, "bound": "valu",
                         "pipe": {"fv": "FP64 VALU (forward FMA + Viterbi add+max pairs)",
                                  "vit": "FP64 VALU (add+max pairs)"}.get(args.mode,
                                                                        "FP64 VALU FMA"),
                         "achieved": round(achieved, 4), "peak": round(dom_peak, 3),
                         "unit": "TFLOP/s", "frac": round(achieved / dom_peak, 5),
                         "peak_source": "AMD spec: FP64 78.6 TFLOP/s (FMA), 39.3 T add/max "
                                        "ops/s",
                         "peak_spec_tflops": FP64_SPEC_TFLOPS,
                         "peak_spec_add_max_tops": FP64_SPEC_ADDMAX_TOPS,
                         "frac_vs_measured_peaks": round(ideal_meas_ms / dom_ms, 5)
                         if dom_ms else None,
                         "measured_peaks": {"fma_tflops": round(fma_meas, 3),
                                            "add_max_tops": round(am_meas, 3),
                                            "source": peak_src},
                         "traffic": traffic, "traffic_note": traffic_note,
                         "kernel_ms": round(dom_ms, 4),
                         "kernel_ms_source": ("HIP events of the timed call in the timed loop "
                                              f"({len(loop_ms)} steps)") if loop_ms else
                                             "HIP events, separate instrumented passes",
                         "forward_ms": round(fwd_avg, 4),
                         "viterbi_ms": round(vit_avg, 4) if args.mode in ("fv", "vit") else None,
                         "traceback_ms": round(tb_avg, 4) if args.mode in ("fv", "vit") else None,
                         "forward_viterbi_ms": round(float(np.mean(fv_ms)), 4) if fv_ms else None,
                         "algorithmic": f"{pair_ops:.0f} FP64 ops/column per sweep x "
                                        f"{cols_local} columns (rank 0)",
                         "step_ideal_ms": round(ideal_ms, 4),
                         "step_frac": round(ideal_ms / step_ms, 5) if not opt_mode else None},
            "cpu_baseline": cpu,
            **({"counters": {"source": rates_src, "kernels": rates}} if rates else {}),
            **({"build_ms": round(float(np.mean(build_ms)), 1)} if opt_mode else {}),
            **({"per_rank_step_ms": per_rank_ms, "allreduce_ms": xchg_ms,
                "allreduce_bytes": int(d_ll_global.numel() * 8)} if dist_on else {}),
            # optimize mode with a split build: each rank's own step still contains the
            # build's all_gather, so it waits for the slowest rank's share of the build
            **({"per_rank_includes": "model build incl. its all_gather (split_build)"}
               if world > 1 and opt_mode and args.backend == "nccl" and args.split_build == 1
               else {}),
            **({"host_path": host} if host is not None else {}),
            **({"shard_projection": shards} if shards is not None else {}),
            **(check or {}),
            "loglik_total": ll_total if args.mode not in ("posterior", "vit") else None,
            "gen_seconds": round(gen_s, 2),
        }
        print(json.dumps(result), flush=True)
    if dist_on:
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
                    f"D2H and float64 outputs included (best of {reps})"}


if __name__ == "__main__":
    main()
