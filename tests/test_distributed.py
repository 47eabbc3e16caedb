"""Block sharding + log-likelihood exchange (itrails_amd/distributed.py) on CPU: gloo,
world size 2 (and 3), the per-shard compute injected as the oracle so the test checks the
sharding and the exchange, not the kernels (those are tests/test_gpu_sweeps.py)."""
import os
import socket

import numpy as np
import pytest

from conftest import ROOT, golden

from itrails_amd.distributed import shard_ranges


def test_shard_ranges_cover_in_order():
    rng = np.random.default_rng(3)
    for world in (1, 2, 3, 8):
        for nb in (0, 1, 2, 5, 37, 400):
            lens = rng.geometric(1 / 500, size=nb)
            if nb > 3:
                lens[rng.integers(0, nb, 3)] = 0  # empty blocks
            r = shard_ranges(lens, world)
            assert len(r) == world
            assert r[0][0] == 0 and r[-1][1] == nb
            for (lo, hi), (lo2, _) in zip(r, r[1:]):
                assert lo <= hi == lo2
            if nb >= 50 * world:
                cols = [int(lens[lo:hi].sum()) for lo, hi in r]
                assert max(cols) - min(cols) <= 2 * lens.max() + 1


def test_shard_ranges_balance_by_columns():
    lens = [10_000] + [10] * 1000  # one long block: rank 0 gets it alone
    r = shard_ranges(lens, 2)
    assert r[0] == (0, 1)


def _oracle_loglik(a, b, pi, V_lst):
    from itrails_amd.tables import build_tables
    from itrails_amd.hmm import concat_blocks
    from oracle import hmm_oracle as O
    if not V_lst:
        return np.zeros(0)
    obs, off = concat_blocks(V_lst)
    return O.forward_loglik(build_tables(a, b, pi), obs, off)


def _worker(rank, world, port, q):
    import sys
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import torch.distributed as dist
    os.environ["OMP_NUM_THREADS"] = "1"
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                            world_size=world)
    try:
        from itrails_amd.distributed import sharded_loglik, local_blocks
        g = golden("sweep_syn27.npz")
        a, b, pi = g["a"], g["b"], g["pi"]
        obs, off = g["obs"], g["off"]
        V_lst = [obs[off[k]:off[k + 1]].astype(np.int64) for k in range(len(off) - 1)]
        tot = sharded_loglik(a, b, pi, V_lst, compute=_oracle_loglik)
        lo, hi, _ = local_blocks(V_lst)
        q.put((rank, tot, lo, hi))
    finally:
        dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_loglik_gloo_matches_block_order_sum(world):
    import torch.multiprocessing as mp
    from itrails_amd.hmm import concat_blocks  # noqa: F401  (import check)
    from oracle import hmm_oracle as O  # noqa: F401
    O.lib()  # build once before forking

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    g = golden("sweep_syn27.npz")
    # single-process reference: the block-order sum of the golden per-block values
    acc = 0.0
    for v in g["loglik"].tolist():
        acc += v
    tots = {r: t for r, t, _, _ in res}
    assert len(set(tots.values())) == 1, "ranks disagree"
    assert abs(tots[0] - acc) <= 1e-12 * abs(acc)
    ranges = sorted((lo, hi) for _, _, lo, hi in res)
    assert ranges[0][0] == 0 and ranges[-1][1] == len(g["off"]) - 1


def test_sharded_sampling_independent_of_world_size():
    """bench.py's strong-scaling workload: every rank samples only its own shard
    (sample_alignment_range), and the union over ranks is the same alignment at every
    world size."""
    from itrails_amd.synth import block_lengths, sample_alignment_range
    g = golden("sweep_syn13.npz")
    a, b, pi = g["a"], g["b"], g["pi"]
    lengths = block_lengths(np.random.default_rng(1), 300_000, 400.0)
    ref = None
    for world in (1, 2, 3, 8):
        parts = []
        for lo, hi in shard_ranges(lengths, world):
            obs, off = sample_alignment_range(a, b, pi, lengths, lo, hi, seed=5, chunk=64)
            assert off[-1] == len(obs) == lengths[lo:hi].sum()
            parts.append(obs)
        allobs = np.concatenate(parts)
        if ref is None:
            ref = allobs
        assert np.array_equal(allobs, ref)
    assert len(ref) == 300_000


def _split_build_worker(rank, world, port, q):
    import sys
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import torch.distributed as dist
    os.environ["OMP_NUM_THREADS"] = "1"
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                            world_size=world)
    try:
        from helpers.torch_linalg import FakeTorchLinalg
        from itrails_amd.model import trans_emiss_calc
        g = golden("model_kat_3_3.npz")
        la = FakeTorchLinalg()
        la.rank, la.world = rank, world
        a, _, pi, _, _ = trans_emiss_calc(*g["args"], 3, 3, la=la)
        q.put((rank, a, pi, la.stats["vanloan"]))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3, 8])
def test_split_model_build_gloo_matches_single_rank(world):
    """The rank-split model build (chains._interval_mats_split: propagators and path groups
    cut into runs of equal Van Loan member cost, one run per rank, one all-gather) gives
    every rank the single-rank model bit for bit; each path is evaluated on exactly one rank
    and every rank's member cost is within 1.3x of the mean."""
    import torch.multiprocessing as mp
    from helpers.torch_linalg import FakeTorchLinalg
    from itrails_amd.model import chains, trans_emiss_calc
    g = golden("model_kat_3_3.npz")
    la = FakeTorchLinalg()
    a1, _, pi1, _, _ = trans_emiss_calc(*g["args"], 3, 3, la=la)
    plan = chains._LAST_PLAN[3]
    (tab,) = plan.dev.values()
    parts = chains.split_partition(plan, tab, world)
    costs = np.array([c for _, c in parts])
    assert costs.max() <= 1.3 * costs.mean(), costs
    units = [u for pu, _ in parts for u in pu]
    assert sorted(units) == sorted(set(units)) and len(units) == sum(
        1 + len(ip.groups) for ip in plan.intervals)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_split_build_worker, args=(r, world, port, q))
             for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in procs]
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    for _, a, pi, _ in res:
        assert np.array_equal(a, a1) and np.array_equal(pi, pi1)
    assert sum(v for _, _, _, v in res) == la.stats["vanloan"]


def test_split_partition_balanced_at_7_intervals():
    """Config 5's (7,7) chain plan over 2..8 ranks: every rank's member cost within 1.3x of
    the mean (the old interval-mod-world split left 2 of 8 ranks idle)."""
    from helpers.torch_linalg import FakeTorchLinalg
    from itrails_amd.model import chains, trans_emiss_calc
    g = golden("model_kat_3_3.npz")
    la = FakeTorchLinalg()
    trans_emiss_calc(*g["args"], 7, 7, la=la)
    plan = chains._LAST_PLAN[7]
    (tab,) = plan.dev.values()
    for world in (2, 4, 8):
        costs = np.array([c for _, c in chains.split_partition(plan, tab, world)])
        assert costs.max() <= 1.3 * costs.mean(), (world, costs)
        # members shared by groups on two ranks are formed twice: the largest rank's cost
        # stays within 1.25x of an even split of the one-rank work
        one = chains.split_partition(plan, tab, 1)[0][1]
        assert costs.max() <= 1.25 * one / world, (world, costs, one)
