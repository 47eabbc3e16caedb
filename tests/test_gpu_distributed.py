"""Multi-rank decoding on the real HIP path: two gloo ranks sharing cuda:0 (the one-GPU box
has a single device; RCCL refuses two ranks on one GPU, gloo carries the same exchange).

* sharded_loglik / sharded_viterbi (itrails_amd/distributed.py, the reference's joblib fan-out
  optimizer.py:40-65 re-shaped as contiguous column-balanced shards) with the default HIP
  compute: the all-reduced block-order total is bit-identical to the single-process
  loglik_wrapper, and the concatenated per-rank paths equal the single-process paths.
* bench.py --gpus 2 launching its own two ranks (no torchrun) on the strong-scaling
  workload: the JSON line reports world size 2, Viterbi paths equal to the CPU restatement
  and log-likelihoods within 1e-8.
"""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

from conftest import ROOT, golden

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _alignment():
    from itrails_amd.synth import block_lengths, sample_alignment
    g = golden("model_kat_5_5.npz")
    a, b, pi = g["a"], g["b"], g["pi"]
    lengths = block_lengths(np.random.default_rng(4), 600_000, 1500.0)
    obs, off, _ = sample_alignment(a, b, pi, lengths, seed=11)
    V = [obs[off[k]:off[k + 1]].astype(np.int64) for k in range(len(off) - 1)]
    return a, b, pi, V


def _worker(rank, world, port, q):
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import torch
    import torch.distributed as dist
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                           world_size=world)
    try:
        from itrails_amd.distributed import sharded_loglik, sharded_viterbi
        a, b, pi, V = _alignment()
        tot = sharded_loglik(a, b, pi, V)
        lo, paths = sharded_viterbi(a, b, pi, V)
        q.put((rank, tot, lo, [np.asarray(p, dtype=np.uint8) for p in paths]))
    finally:
        dist.destroy_process_group()


def test_two_ranks_hip_bit_identical_to_single_rank(gpu):
    import torch.multiprocessing as mp
    from itrails_amd import hmm

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted((q.get(timeout=240) for _ in procs), key=lambda r: r[0])
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    a, b, pi, V = _alignment()
    single = hmm.loglik_wrapper(a, b, pi, V)
    paths = hmm.viterbi_wrapper(a, b, pi, V)
    assert res[0][1] == res[1][1] == single  # bit-identical block-order total
    lo0, lo1 = res[0][2], res[1][2]
    assert lo0 == 0 and 0 < lo1 < len(V)
    got = np.concatenate(res[0][3] + res[1][3])
    np.testing.assert_array_equal(got, np.concatenate(paths).astype(np.uint8))


def test_bench_self_launch_two_ranks(gpu):
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--backend", "gloo",
           "--workload", "chr100", "--mbp", "3", "--steps", "2", "--warmup", "1",
           "--host-path", "0"]
    out = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=600)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout
    r = json.loads(lines[0])
    assert r["n_gpus"] == 2 and r["config"]["world_size_seen"] == 2
    assert r["scaling"] == "strong" and r["config"]["columns_total"] == 3_000_000
    assert r["viterbi_equal"] is True and r["columns_checked"] == 3_000_000
    assert r["loglik_max_rel_err"] < 1e-8


def _split_worker(rank, world, port, q):
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import torch
    import torch.distributed as dist
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                            world_size=world)
    try:
        from itrails_amd.model import trans_emiss_calc
        from itrails_amd.model.linalg import DeviceLinalg, split_build
        g = golden("model_kat_5_5.npz")
        with split_build(True):
            la = DeviceLinalg()
            a, b, pi, _, _ = trans_emiss_calc(*g["args"], 5, 5, la=la)
        q.put((rank, a, pi, la.stats["vanloan"]))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_split_model_build_ranks_match_single_rank(gpu, world):
    """The rank-split (5,5) model build on the real HIP path (gloo ranks on cuda:0): each
    rank evaluates its run of the propagators and path groups (chains.split_partition;
    intervals cut mid-way, each interval's Pade branch fixed by the norms of all its paths),
    the all-gather shares them, and every rank's model equals the single-rank build bit for
    bit (and the reference's within the model tolerance)."""
    import torch.multiprocessing as mp
    from itrails_amd.model import trans_emiss_calc
    from itrails_amd.model.linalg import DeviceLinalg
    g = golden("model_kat_5_5.npz")
    la = DeviceLinalg()
    a1, _, pi1, _, _ = trans_emiss_calc(*g["args"], 5, 5, la=la)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_split_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in procs]
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    for _, a, pi, _ in res:
        assert np.array_equal(a, a1) and np.array_equal(pi, pi1)
        assert np.allclose(a, g["a"], rtol=1e-10, atol=1e-15)
    assert sum(v for _, _, _, v in res) == la.stats["vanloan"]


def test_rccl_world1_beside_partition_streams(gpu):
    """RCCL (the `nccl` backend) executing on this one GPU beside itr_forward_viterbi's three
    CU-masked streams, with the queue setting bench.py uses for N > 1
    (GPU_MAX_HW_QUEUES = 8): bench.py --dist 1 initialises a world-size-1 nccl group, so
    every timed step's log-likelihood exchange is a real all-reduce of the per-block vector
    after the partitioned sweep; the line must report the nccl backend, the exchange time,
    Viterbi paths equal to the CPU restatement and log-likelihoods within 1e-8."""
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT"):
        env.pop(k, None)
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "1", "--dist", "1",
           "--backend", "nccl", "--mbp", "2", "--steps", "3", "--warmup", "2",
           "--host-path", "0", "--cpu-1core-cols", "0"]
    out = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout
    r = json.loads(lines[0])
    assert r["config"]["backend"] == "nccl" and r["config"]["world_size_seen"] == 1
    assert r["allreduce_ms"] is not None and r["allreduce_ms"] > 0
    assert r["viterbi_equal"] is True and r["columns_checked"] == 2_000_000
    assert r["loglik_max_rel_err"] < 1e-8
