"""The hot path at BASELINE.json's full size (config 2: the (5,5) model, 10 Mbp in geometric
blocks of mean 2 kbp, 5,036 blocks, longest 18,377 columns) checked through properties that
do not need the CPU oracle to run over all of it:

  * the longest blocks (which the forward sweep splits into a forward and a backward half,
    meet in the middle) and a seeded sample of the rest against the oracle: log-likelihoods
    within 1e-8 relative, Viterbi paths identical;
  * the split forward against the unsplit one on every split block (split_frac=0 at plan
    creation): the same value to 1e-12 relative;
  * the combined call the bench times (itr_forward_viterbi: the CU-partitioned forward +
    Viterbi) against the oracle on EVERY block: paths identical, log-likelihoods 1e-8; and
    the same on every one of BASELINE config 4's eight shards at world size 8 (the chr100
    layout, which takes the other branches of the partition);
  * the device-built (5,5) model against the reference-built one on the whole workload;
  * every block's log-likelihood finite and negative, the total equal to the block-order
    sum of the per-block values (loglik_wrapper semantics);
  * every posterior row sums to 1 (1e-12) and matches the oracle (1e-8), every block;
  * BASELINE config 3 (the reference's (7,7) model, N = 133) and the introgression (5,5)
    model (N = 95) against the oracle on every block: posterior rows 1e-8, Viterbi paths
    identical, log-likelihoods 1e-8.
"""
import os

import numpy as np
import pytest

from conftest import golden
from itrails_amd import hmm
from itrails_amd.synth import block_lengths, sample_alignment
from itrails_amd.tables import build_tables
from oracle import hmm_oracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def full(gpu):
    import torch
    g = golden("model_kat_5_5.npz")
    a, b, pi = g["a"], g["b"], g["pi"]
    rng = np.random.default_rng(12345)  # bench.py's layout
    lengths = block_lengths(rng, 10_000_000, 2000.0)
    obs, off, _ = sample_alignment(a, b, pi, lengths, seed=777)
    model, plan = hmm.Model(a, b, pi), hmm.Plan(off)
    d_obs = torch.from_numpy(obs.astype(np.int16)).cuda()
    ll = hmm.forward_loglik_device(model, plan, d_obs).cpu().numpy()
    path = hmm.viterbi_device(model, plan, d_obs).cpu().numpy()
    lens = np.diff(off)
    srng = np.random.default_rng(5)
    longest = np.argsort(-lens, kind="stable")[:12]
    sample = np.unique(np.concatenate([longest, srng.choice(len(lens), 60, replace=False)]))
    return dict(a=a, b=b, pi=pi, obs=obs, off=off, model=model, d_obs=d_obs, ll=ll,
                path=path, sample=sample, longest=longest, t=build_tables(a, b, pi))


def _sub(obs, off, blocks):
    parts = [obs[off[k]:off[k + 1]] for k in blocks]
    sub_off = np.zeros(len(blocks) + 1, dtype=np.int64)
    sub_off[1:] = np.cumsum([len(p) for p in parts])
    return np.concatenate(parts), sub_off


def test_full_size_layout(full):
    assert full["off"][-1] == 10_000_000
    assert len(full["off"]) - 1 == 5036
    assert np.diff(full["off"]).max() == 18377


def test_full_size_sample_vs_oracle(full):
    obs, off, sample = full["obs"], full["off"], full["sample"]
    so, soff = _sub(obs, off, sample)
    ll_ref = O.forward_loglik(full["t"], so, soff)
    np.testing.assert_allclose(full["ll"][sample], ll_ref, rtol=1e-8, atol=0)
    path_ref = O.viterbi(full["t"], so, soff)
    got = np.concatenate([full["path"][off[k]:off[k + 1]] for k in sample])
    np.testing.assert_array_equal(got, path_ref)


def test_full_size_split_forward_matches_unsplit(full):
    plan = hmm.Plan(full["off"], split_frac=0)
    ll = hmm.forward_loglik_device(full["model"], plan, full["d_obs"]).cpu().numpy()
    k = full["longest"]
    np.testing.assert_allclose(full["ll"][k], ll[k], rtol=1e-12, atol=0)
    np.testing.assert_allclose(full["ll"], ll, rtol=1e-12, atol=0)


def _check_all_blocks(t, obs, off, ll, path):
    ll_ref = O.forward_loglik(t, obs, off)
    np.testing.assert_allclose(ll, ll_ref, rtol=1e-8, atol=0)
    path_ref = O.viterbi(t, obs, off)
    bad = np.flatnonzero(path != path_ref)
    assert bad.size == 0, f"{bad.size} columns differ, first at {bad[:5]}"


def test_full_size_forward_viterbi_every_block(full):
    """BASELINE config 2 exactly as bench.py times it: itr_forward_viterbi over all 10 M
    columns (forward halves on reserved CUs beside the Viterbi long blocks, the per-wave
    Viterbi on the others) against the CPU restatement on every block."""
    plan = hmm.Plan(full["off"])
    ll, path = hmm.forward_viterbi_device(full["model"], plan, full["d_obs"])
    ll, path = ll.cpu().numpy(), path.cpu().numpy()
    assert np.array_equal(path, full["path"])  # the separate calls' paths, bit for bit
    np.testing.assert_allclose(ll, full["ll"], rtol=1e-12, atol=0)
    _check_all_blocks(full["t"], full["obs"], full["off"], ll, path)


@pytest.mark.parametrize("prune", [0, 1 << 62])
def test_full_size_viterbi_either_step(full, prune):
    """The per-wave Viterbi with every bulk block on the full scan, and on the bound-pruned
    step (itr_plan_set_prune_len): the same 10 M-column path, bit for bit, as the planned mix
    (checked against the CPU restatement on every block above)."""
    plan = hmm.Plan(full["off"])
    plan.set_prune_len(prune)
    _, path = hmm.forward_viterbi_device(full["model"], plan, full["d_obs"])
    assert np.array_equal(path.cpu().numpy(), full["path"])
    path = hmm.viterbi_device(full["model"], plan, full["d_obs"])
    assert np.array_equal(path.cpu().numpy(), full["path"])


@pytest.mark.parametrize("rank", range(8))
def test_chr100_shard_forward_viterbi(gpu, rank):
    """BASELINE config 4's per-rank work at world size 8: every shard of the fixed 100 Mbp
    alignment (bench.py --workload chr100: shard_ranges over the geometric block layout,
    ~12.5 Mbp each; rank 3 holds the alignment's longest block, 23,881 columns) through
    itr_forward_viterbi, every block against the oracle."""
    import torch
    from itrails_amd.distributed import shard_ranges
    from itrails_amd.synth import sample_alignment_range
    g = golden("model_kat_5_5.npz")
    a, b, pi = g["a"], g["b"], g["pi"]
    lengths = block_lengths(np.random.default_rng(12345), 100_000_000, 2000.0)
    lo, hi = shard_ranges(lengths, 8)[rank]
    obs, off = sample_alignment_range(a, b, pi, lengths, lo, hi, seed=777)
    assert 11_000_000 < off[-1] < 14_000_000
    if rank == 3:
        assert np.diff(off).max() == lengths.max() == 23881
    model, plan = hmm.Model(a, b, pi), hmm.Plan(off)
    d_obs = torch.from_numpy(obs.astype(np.int16)).cuda()
    ll, path = hmm.forward_viterbi_device(model, plan, d_obs)
    _check_all_blocks(build_tables(a, b, pi), obs, off, ll.cpu().numpy(), path.cpu().numpy())
    del d_obs, plan
    torch.cuda.empty_cache()


def test_device_built_vs_reference_model_decode(full):
    """config 2 decoded with the (5,5) model the drop-in CLIs build on the
    device (model.trans_emiss_calc, KAT parameters) instead of the reference-built one
    (tests/golden/model_kat_5_5.npz).  The two models agree to ~1e-15 (a, pi) / 1e-8 (b);
    the log-likelihoods agree within 1e-8 relative; the number of Viterbi columns that differ
    is recorded, not asserted zero: a near-tie decided by the last bit can
    flip."""
    import json
    from itrails_amd.model import trans_emiss_calc
    from itrails_amd.model.linalg import DeviceLinalg
    g = golden("model_kat_5_5.npz")
    n_ab, n_abc = (int(x) for x in g["n_int"])
    a, b, pi, _, _ = trans_emiss_calc(*g["args"], n_ab, n_abc, la=DeviceLinalg())
    model = hmm.Model(a, b, pi)
    plan = hmm.Plan(full["off"])
    ll, path = hmm.forward_viterbi_device(model, plan, full["d_obs"])
    ll, path = ll.cpu().numpy(), path.cpu().numpy()
    np.testing.assert_allclose(ll, full["ll"], rtol=1e-8, atol=0)
    diff = int((path != full["path"]).sum())
    rel = float(np.max(np.abs(ll - full["ll"]) / np.abs(full["ll"])))
    print(json.dumps({"viterbi_columns_differing": diff, "columns": int(full["off"][-1]),
                      "loglik_max_rel_diff": rel, "a_max_abs_diff": float(np.abs(a - g["a"]).max()),
                      "b_max_abs_diff": float(np.abs(b - g["b"]).max())}))
    assert diff <= 1000  # (observed: see DESIGN.md §7)


def test_full_size_loglik_properties(full):
    ll = full["ll"]
    assert np.isfinite(ll).all() and (ll < 0).all()
    acc = 0.0
    for v in ll.tolist():
        acc += v
    V = [full["obs"][full["off"][k]:full["off"][k + 1]].astype(np.int64)
         for k in range(len(full["off"]) - 1)]
    assert hmm.loglik_wrapper(full["a"], full["b"], full["pi"], V) == acc


def test_full_size_posterior_rows(full):
    import torch
    plan = hmm.Plan(full["off"])
    plan.reserve(full["a"].shape[0], posterior=True)
    post = hmm.posterior_device(full["model"], plan, full["d_obs"])
    sums = post.sum(dim=1)
    assert float((sums - 1.0).abs().max()) < 1e-12
    assert _posterior_every_block(full["t"], full["obs"], full["off"], post) == 10_000_000
    del post
    torch.cuda.empty_cache()


def test_full_size_posterior_split_matches_unsplit(full):
    """The posterior's concurrent forward/backward split (the longest blocks' backward
    sweeps run beside the forward sweep, post_combine_kernel joins the stored rows) against
    the two-pass sweep (post_split_frac=0 at plan creation) on every row, and the
    longest blocks against the CPU restatement."""
    import torch
    n = full["a"].shape[0]
    plan = hmm.Plan(full["off"])
    plan.reserve(n, posterior=True)
    post = hmm.posterior_device(full["model"], plan, full["d_obs"])
    plan0 = hmm.Plan(full["off"], post_split_frac=0)
    plan0.reserve(n, posterior=True)
    post0 = hmm.posterior_device(full["model"], plan0, full["d_obs"])
    assert float((post - post0).abs().max()) < 1e-12
    del post0, plan0
    obs, off, k = full["obs"], full["off"], np.sort(full["longest"][:3])
    so, soff = _sub(obs, off, k)
    ref = O.posterior(full["t"], so, soff)
    rows = torch.cat([post[off[b]:off[b + 1]] for b in k]).cpu().numpy()
    np.testing.assert_allclose(rows, ref, rtol=1e-8, atol=1e-300)
    del post
    torch.cuda.empty_cache()


def test_full_size_posterior_host_copy(full):
    """post_prob_wrapper from host blocks (itr_posterior_host: 5.6 GB of rows returned
    through the chunked pinned-staging copy) equals the device-resident posterior bit for
    bit, including the partial last chunk."""
    import torch
    obs, off = full["obs"], full["off"]
    nb = int(np.searchsorted(off, 2_000_000))  # ~2 Mbp: 1.1 GB of rows, 9 chunks
    V = [obs[off[k]:off[k + 1]].astype(np.int64) for k in range(nb)]
    host = hmm.post_prob_wrapper(full["a"], full["b"], full["pi"], V)
    plan = hmm.Plan(off[:nb + 1])
    plan.reserve(full["a"].shape[0], posterior=True)
    post = hmm.posterior_device(full["model"], plan, full["d_obs"][:off[nb]]).cpu().numpy()
    assert len(host) == nb and all(h.shape == (len(v), 70) for h, v in zip(host, V))
    assert np.array_equal(np.concatenate(host), post)
    del post, host
    torch.cuda.empty_cache()


# ---------------------------------------------------------------------------------------
# BASELINE config 3: the reference's own (7,7) model (N = 133, tests/golden/model_kat_7_7.npz,
# 3,638 s of reference build), 10 Mbp, posterior decoding (+ forward and Viterbi)
# ---------------------------------------------------------------------------------------
@pytest.fixture(scope="module")
def full77(gpu):
    import torch
    g = golden("model_kat_7_7.npz")
    a, b, pi = g["a"], g["b"], g["pi"]
    rng = np.random.default_rng(12345)  # bench.py's layout
    lengths = block_lengths(rng, 10_000_000, 2000.0)
    obs, off, _ = sample_alignment(a, b, pi, lengths, seed=777)
    model, plan = hmm.Model(a, b, pi), hmm.Plan(off)
    d_obs = torch.from_numpy(obs.astype(np.int16)).cuda()
    lens = np.diff(off)
    longest = np.argsort(-lens, kind="stable")[:6]
    sample = np.unique(np.concatenate([longest, np.random.default_rng(6).choice(len(lens), 24,
                                                                                replace=False)]))
    return dict(a=a, b=b, pi=pi, obs=obs, off=off, model=model, plan=plan, d_obs=d_obs,
                sample=sample, t=build_tables(a, b, pi))


def _posterior_every_block(t, obs, off, post, chunk_cols=1_000_000):
    """Every posterior row of a device posterior `post` (total x N, on the device) against
    the CPU restatement, in runs of whole blocks of about chunk_cols columns so host memory
    stays bounded (10 Mbp x 133 states is 10.6 GB of rows): rows to 1e-8 relative."""
    nb = len(off) - 1
    k0, checked = 0, 0
    while k0 < nb:
        k1 = int(np.searchsorted(off, off[k0] + chunk_cols, side="right")) - 1
        k1 = min(nb, max(k0 + 1, k1))
        o = off[k0:k1 + 1] - off[k0]
        ref = O.posterior(t, obs[off[k0]:off[k1]], o)
        rows = post[off[k0]:off[k1]].cpu().numpy()
        np.testing.assert_allclose(rows, ref, rtol=1e-8, atol=1e-300,
                                   err_msg=f"blocks {k0}..{k1 - 1}")
        checked += rows.shape[0]
        k0 = k1
    return checked


def test_full_size_77_posterior(full77):
    """BASELINE config 3 in full: every posterior row of the 10 Mbp alignment (all 5,036
    blocks) against the CPU restatement to 1e-8 relative, and every row sums to 1 (1e-12)."""
    import torch
    f = full77
    f["plan"].reserve(133, posterior=True)
    post = hmm.posterior_device(f["model"], f["plan"], f["d_obs"])
    assert float((post.sum(dim=1) - 1.0).abs().max()) < 1e-12
    assert _posterior_every_block(f["t"], f["obs"], f["off"], post) == 10_000_000
    del post
    torch.cuda.empty_cache()


def test_full_size_77_forward_viterbi(full77):
    """Config 3's model through both decoding calls, every block against the CPU
    restatement: the separate forward / Viterbi calls and the combined itr_forward_viterbi
    (paths identical on all 10 M columns, log-likelihoods 1e-8)."""
    f = full77
    ll = hmm.forward_loglik_device(f["model"], f["plan"], f["d_obs"]).cpu().numpy()
    path = hmm.viterbi_device(f["model"], f["plan"], f["d_obs"]).cpu().numpy()
    assert np.isfinite(ll).all() and (ll < 0).all()
    _check_all_blocks(f["t"], f["obs"], f["off"], ll, path)
    ll2, path2 = hmm.forward_viterbi_device(f["model"], f["plan"], f["d_obs"])
    assert np.array_equal(path2.cpu().numpy(), path)
    np.testing.assert_allclose(ll2.cpu().numpy(), ll, rtol=1e-12, atol=0)


# ---------------------------------------------------------------------------------------
# the introgression (5,5) model (N = 95, the reference's own build,
# tests/golden/model_int_ikat_5_5.npz) over the full 10 Mbp layout
# ---------------------------------------------------------------------------------------
def test_full_size_intro95_every_block(gpu):
    """itrails-int-viterbi's hot path at N = 95 over 10 Mbp (5,036 blocks): forward
    log-likelihoods (1e-8) and Viterbi paths (identical) of every block against the CPU
    restatement, through the combined call and the Viterbi-only call; the posterior rows
    of the first ~1 Mbp against the restatement (1e-8) and every row summing to 1."""
    import torch
    g = golden("model_int_ikat_5_5.npz")
    a, b, pi = g["a"], g["b"], g["pi"]
    assert a.shape[0] == 95
    lengths = block_lengths(np.random.default_rng(12345), 10_000_000, 2000.0)
    obs, off, _ = sample_alignment(a, b, pi, lengths, seed=777)
    t = build_tables(a, b, pi)
    model, plan = hmm.Model(a, b, pi), hmm.Plan(off)
    d_obs = torch.from_numpy(obs.astype(np.int16)).cuda()
    ll, path = hmm.forward_viterbi_device(model, plan, d_obs)
    ll, path = ll.cpu().numpy(), path.cpu().numpy()
    _check_all_blocks(t, obs, off, ll, path)
    assert np.array_equal(hmm.viterbi_device(model, plan, d_obs).cpu().numpy(), path)
    nb = int(np.searchsorted(off, 1_000_000))
    sub = hmm.Plan(off[:nb + 1])
    sub.reserve(95, posterior=True)
    post = hmm.posterior_device(model, sub, d_obs[:off[nb]])
    assert float((post.sum(dim=1) - 1.0).abs().max()) < 1e-12
    assert _posterior_every_block(t, obs[:off[nb]], off[:nb + 1], post) == off[nb]
    del post, d_obs
    torch.cuda.empty_cache()


def test_short_blocks_133_pruned_viterbi(gpu):
    """The bound-pruned Viterbi (prune_vit.hip: one block per wavefront, log a in LDS), which
    itr_viterbi / itr_forward_viterbi take at N = 133 for many short blocks: 2 Mbp of the
    (7,7) model in geometric blocks of mean 300 columns, every path against the CPU
    restatement, the log-likelihoods of the combined call 1e-8."""
    import torch
    g = golden("model_kat_7_7.npz")
    a, b, pi = g["a"], g["b"], g["pi"]
    lengths = block_lengths(np.random.default_rng(1), 2_000_000, 300.0)
    obs, off, _ = sample_alignment(a, b, pi, lengths, seed=778)
    assert len(lengths) > 2 * 256 and off[-1] / len(lengths) <= 400  # (the kernel's regime)
    model, plan = hmm.Model(a, b, pi), hmm.Plan(off)
    d_obs = torch.from_numpy(obs.astype(np.int16)).cuda()
    path = hmm.viterbi_device(model, plan, d_obs).cpu().numpy()
    ll, path2 = hmm.forward_viterbi_device(model, plan, d_obs)
    assert np.array_equal(path2.cpu().numpy(), path)
    _check_all_blocks(build_tables(a, b, pi), obs, off, ll.cpu().numpy(), path)


@pytest.mark.parametrize("golden_name,n", [("model_kat_5_5.npz", 70), ("model_kat_7_7.npz", 133)])
def test_hybrid_posterior_split_blocks(gpu, golden_name, n):
    """The matrix-core posterior's split of its longest blocks (itr_posterior: a beta-only
    sweep over [lo, T) beside the forward launch, the backward launch's VALU task over
    [0, lo] from the stored beta_lo, post_combine for (lo, T)) at N = 70 and N = 133, on a
    mid-size layout: four long blocks (VALU tasks, split) among 700 short ones (matrix-core
    groups; more than two blocks per CU, so the VALU-only concurrent split does not take
    it).  Every row against the CPU restatement (1e-8) and against the same plan without
    the split (post_split_frac=0: the long blocks' whole backward + posterior sweep in the
    backward launch), 1e-12."""
    import torch
    g = golden(golden_name)
    a, b, pi = g["a"], g["b"], g["pi"]
    assert a.shape[0] == n
    short = block_lengths(np.random.default_rng(21), 210_000, 300.0)
    lengths = np.concatenate([[6000, 5200, 4700, 5600], short]).astype(np.int64)
    obs, off, _ = sample_alignment(a, b, pi, lengths, seed=901)
    assert len(lengths) > 2 * 256 + 4
    model = hmm.Model(a, b, pi)
    d_obs = torch.from_numpy(obs.astype(np.int16)).cuda()
    plan = hmm.Plan(off)
    plan.reserve(n, posterior=True)
    post = hmm.posterior_device(model, plan, d_obs)
    plan0 = hmm.Plan(off, post_split_frac=0)
    plan0.reserve(n, posterior=True)
    post0 = hmm.posterior_device(model, plan0, d_obs)
    np.testing.assert_allclose(post.cpu().numpy(), post0.cpu().numpy(), rtol=1e-12, atol=1e-300)
    assert float((post.sum(dim=1) - 1.0).abs().max()) < 1e-12
    t = build_tables(a, b, pi)
    assert _posterior_every_block(t, obs, off, post, chunk_cols=100_000) == off[-1]
    del post, post0, d_obs
    torch.cuda.empty_cache()


@pytest.mark.parametrize("n", [137, 141])
def test_short_blocks_pruned_viterbi_layout_limits(gpu, n):
    """N = 137 and 141 in the pruned Viterbi's regime (many short blocks): its layout holds
    only two blocks per CU beside the matrix at N = 137 and does not fit the 160 KiB of LDS
    at N = 141, so itr_viterbi / itr_forward_viterbi must take the 9-wave layout instead of
    failing the launch; every path against the CPU restatement."""
    import torch
    from test_gpu_sweeps import random_hmm
    a, b, pi = random_hmm(np.random.default_rng(n), n)
    lengths = block_lengths(np.random.default_rng(2), 200_000, 300.0)
    obs, off, _ = sample_alignment(a, b, pi, lengths, seed=n)
    assert len(lengths) > 2 * 256 and off[-1] / len(lengths) <= 400
    model, plan = hmm.Model(a, b, pi), hmm.Plan(off)
    d_obs = torch.from_numpy(obs.astype(np.int16)).cuda()
    path = hmm.viterbi_device(model, plan, d_obs).cpu().numpy()
    ll, path2 = hmm.forward_viterbi_device(model, plan, d_obs)
    assert np.array_equal(path2.cpu().numpy(), path)
    _check_all_blocks(build_tables(a, b, pi), obs, off, ll.cpu().numpy(), path)


def test_full_size_n27_every_block(gpu):
    """The reference's example workload (it/examples/example_config.yaml:19-20:
    n_int_AB = n_int_ABC = 3, N = 27 hidden states; the reference's own (3,3) build,
    tests/golden/model_kat_3_3.npz) over the config-2 layout (10 Mbp, 5,036 blocks): forward
    log-likelihoods (1e-8) and Viterbi paths (identical) of every block through the combined
    and the Viterbi-only call, and every posterior row (1e-8, rows summing to 1)."""
    import torch
    g = golden("model_kat_3_3.npz")
    a, b, pi = g["a"], g["b"], g["pi"]
    assert a.shape[0] == 27
    lengths = block_lengths(np.random.default_rng(12345), 10_000_000, 2000.0)
    obs, off, _ = sample_alignment(a, b, pi, lengths, seed=777)
    t = build_tables(a, b, pi)
    model, plan = hmm.Model(a, b, pi), hmm.Plan(off)
    d_obs = torch.from_numpy(obs.astype(np.int16)).cuda()
    ll, path = hmm.forward_viterbi_device(model, plan, d_obs)
    ll, path = ll.cpu().numpy(), path.cpu().numpy()
    _check_all_blocks(t, obs, off, ll, path)
    assert np.array_equal(hmm.viterbi_device(model, plan, d_obs).cpu().numpy(), path)
    plan.reserve(27, posterior=True)
    post = hmm.posterior_device(model, plan, d_obs)
    assert float((post.sum(dim=1) - 1.0).abs().max()) < 1e-12
    assert _posterior_every_block(t, obs, off, post) == 10_000_000
    del post, d_obs
    torch.cuda.empty_cache()
