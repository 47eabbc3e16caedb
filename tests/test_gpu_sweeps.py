"""Device sweeps vs the reference (golden vectors) and vs the CPU oracle (larger inputs).

Bars (BASELINE.json north_star): Viterbi paths identical (integer-exact); log-likelihoods
and posteriors within 1e-8 relative.  Posteriors are compared with rtol=1e-8 and
atol=1e-300 (values below ~1e-300 are denormal/underflowed in both computations).
"""
import os

import numpy as np
import pytest

from conftest import golden, int_model_fixtures, model_fixtures, sweep_fixtures
from itrails_amd import hmm
from itrails_amd.synth import sample_alignment
from itrails_amd.tables import build_tables
from oracle import hmm_oracle as O

pytestmark = pytest.mark.gpu

RTOL = 1e-8


def run_all(a, b, pi, obs, off):
    model = hmm.Model(a, b, pi)
    plan = hmm.Plan(off)
    ll = hmm.block_logliks(model, plan, obs)
    path = hmm._paths(model, plan, obs)
    post = hmm._posteriors(model, plan, obs)
    return ll, path, post


def random_hmm(rng, n, stay=(0.9, 0.999)):
    if n == 1:
        return np.ones((1, 1)), rng.dirichlet(np.full(256, 0.3), size=1), np.ones(1)
    a = rng.random((n, n)) ** 3
    np.fill_diagonal(a, 0)
    a /= a.sum(1, keepdims=True)
    d = rng.uniform(*stay, size=n)
    a = a * (1 - d)[:, None]
    a[np.arange(n), np.arange(n)] = d
    b = rng.dirichlet(np.full(256, 0.3), size=n)
    pi = rng.dirichlet(np.ones(n))
    return a, b, pi


EDGE_LENGTHS = [1, 0, 2, 3, 255, 256, 257, 511, 512, 513, 17, 1000, 0, 4096, 1]


@pytest.mark.parametrize("name", sweep_fixtures())
def test_golden_sweeps(gpu, name):
    g = golden(name)
    ll, path, post = run_all(g["a"], g["b"], g["pi"], g["obs"], g["off"])
    np.testing.assert_allclose(ll, g["loglik"], rtol=RTOL, atol=0)
    np.testing.assert_array_equal(path, g["path"])
    np.testing.assert_allclose(post[g["post_rows"]], g["post"], rtol=RTOL, atol=1e-300)


@pytest.mark.parametrize("n", [1, 4, 16, 17, 27, 64, 65, 70, 72, 96, 133, 137, 141, 144, 150, 192])
def test_random_vs_oracle(gpu, n):
    rng = np.random.default_rng(1000 + n)
    a, b, pi = random_hmm(rng, n)
    lengths = EDGE_LENGTHS + list(rng.integers(1, 2500, size=40))
    obs, off, _ = sample_alignment(a, b, pi, lengths, seed=n, p_n=0.03, p_gap=0.02)
    t = build_tables(a, b, pi)
    ll, path, post = run_all(a, b, pi, obs, off)
    np.testing.assert_allclose(ll, O.forward_loglik(t, obs, off), rtol=RTOL, atol=0)
    np.testing.assert_array_equal(path, O.viterbi(t, obs, off))
    np.testing.assert_allclose(post, O.posterior(t, obs, off), rtol=RTOL, atol=1e-300)
    np.testing.assert_allclose(post.sum(1), 1.0, rtol=1e-12)


def test_ties_first_maximum(gpu):
    """Uniform transitions and duplicated emission rows make many exact ties; the device
    must resolve every one to the lowest state like np.argmax (optimizer.py:331,346)."""
    rng = np.random.default_rng(5)
    n = 70
    a = np.full((n, n), 1.0 / n)
    b = rng.dirichlet(np.full(256, 0.5), size=n // 2)
    b = np.repeat(b, 2, axis=0)
    pi = np.full(n, 1.0 / n)
    obs, off, _ = sample_alignment(a, b, pi, [1, 300, 700, 1], seed=9)
    t = build_tables(a, b, pi)
    model, plan = hmm.Model(a, b, pi), hmm.Plan(off)
    np.testing.assert_array_equal(hmm._paths(model, plan, obs), O.viterbi(t, obs, off))


# per-wave Viterbi step choice (itr_plan_set_prune_len): planned lengths, every block on the
# full scan, every block on the bound-pruned step
PRUNE = [None, 0, 1 << 62]


@pytest.mark.parametrize("prune", PRUNE)
@pytest.mark.parametrize("combined", [False, True])
def test_bound_fails_everywhere(gpu, combined, prune):
    """Flat transitions and duplicated emission rows: the per-wave Viterbi's bound test
    (wave_tasks.h) fails for every target of every column, so every column runs all nine
    scan columns, and the exact ties must still resolve to the lowest state.  Hundreds of
    blocks under 2,048 columns, so the per-wave layout takes them (itr_viterbi and
    itr_forward_viterbi), on either step."""
    import torch

    rng = np.random.default_rng(6)
    n = 70
    a = np.full((n, n), 1.0 / n)
    b = np.repeat(rng.dirichlet(np.full(256, 0.5), size=n // 2), 2, axis=0)
    pi = np.full(n, 1.0 / n)
    lengths = [1, 2, 17, 2000] + list(rng.integers(1, 2000, size=300))
    obs, off, _ = sample_alignment(a, b, pi, lengths, seed=11)
    t = build_tables(a, b, pi)
    model, plan = hmm.Model(a, b, pi), hmm.Plan(off)
    plan.set_prune_len(prune)
    d_obs = torch.from_numpy(obs.astype(np.int16)).to(gpu)
    if combined:
        ll, path = hmm.forward_viterbi_device(model, plan, d_obs)
        np.testing.assert_allclose(ll.cpu().numpy(), O.forward_loglik(t, obs, off), rtol=RTOL,
                                   atol=0)
    else:
        path = hmm.viterbi_device(model, plan, d_obs)
    np.testing.assert_array_equal(path.cpu().numpy(), O.viterbi(t, obs, off))


def test_paired_long_set_vs_oracle(gpu):
    """The long Viterbi set swept two blocks per reserved CU (40 blocks of 3,000 columns beside
    2 M columns of short blocks: tests/test_partition.py test_long_set_pairing), through
    itr_forward_viterbi and itr_viterbi, every block against the CPU restatement."""
    import torch

    rng = np.random.default_rng(5)
    lengths = [3000] * 40 + list(rng.integers(100, 600, size=5600))
    g = golden("model_kat_5_5.npz")
    a, b, pi = g["a"], g["b"], g["pi"]
    obs, off, _ = sample_alignment(a, b, pi, lengths, seed=21)
    t = build_tables(a, b, pi)
    model, plan = hmm.Model(a, b, pi), hmm.Plan(off)
    d_obs = torch.from_numpy(obs.astype(np.int16)).to(gpu)
    ref = O.viterbi(t, obs, off)
    ll, path = hmm.forward_viterbi_device(model, plan, d_obs)
    np.testing.assert_array_equal(path.cpu().numpy(), ref)
    np.testing.assert_allclose(ll.cpu().numpy(), O.forward_loglik(t, obs, off), rtol=RTOL, atol=0)
    np.testing.assert_array_equal(hmm.viterbi_device(model, plan, d_obs).cpu().numpy(), ref)


@pytest.mark.parametrize("prune", PRUNE)
@pytest.mark.parametrize("n", [65, 70, 72])
def test_viterbi_zero_probabilities(gpu, n, prune):
    """Zeros in a, b and pi (log 0 = -inf in the Viterbi's sums): unreachable states,
    impossible emissions and targets without any off-diagonal source, at the state counts of
    the per-wave layout, on either step."""
    rng = np.random.default_rng(90 + n)
    a, b, pi = random_hmm(rng, n, stay=(0.5, 0.99))
    a[rng.random((n, n)) < 0.5] = 0.0
    a[:, 3] = 0.0
    a[np.arange(n), np.arange(n)] = 0.5
    a[3, :] = 0.0
    a[3, 3] = 1.0  # state 3: no incoming transitions from other states
    a /= a.sum(1, keepdims=True)
    b[rng.random((n, 256)) < 0.3] = 0.0
    b /= b.sum(1, keepdims=True)
    pi[rng.random(n) < 0.3] = 0.0
    pi /= pi.sum()
    lengths = list(rng.integers(1, 1800, size=200)) + [1, 2, 3000]
    obs, off, _ = sample_alignment(a, b, pi, lengths, seed=n, p_n=0.02, p_gap=0.01)
    t = build_tables(a, b, pi)
    model, plan = hmm.Model(a, b, pi), hmm.Plan(off)
    plan.set_prune_len(prune)
    np.testing.assert_array_equal(hmm._paths(model, plan, obs), O.viterbi(t, obs, off))


@pytest.mark.parametrize("name", [m for m in model_fixtures() if m != "model_kat_1_1.npz"]
                         + int_model_fixtures())
def test_reference_models_vs_oracle(gpu, name):
    """The reference's own model builds (a, b, pi from trans_emiss_calc and from
    trans_emiss_calc_introgression, whose sweeps are the same functions,
    int_optimizer.py:147-380) on sampled data."""
    g = golden(name)
    a, b, pi = g["a"], g["b"], g["pi"]
    rng = np.random.default_rng(3)
    lengths = list(rng.geometric(1 / 1500, size=30)) + [1, 5000]
    obs, off, _ = sample_alignment(a, b, pi, lengths, seed=7)
    t = build_tables(a, b, pi)
    ll, path, post = run_all(a, b, pi, obs, off)
    np.testing.assert_allclose(ll, O.forward_loglik(t, obs, off), rtol=RTOL, atol=0)
    np.testing.assert_array_equal(path, O.viterbi(t, obs, off))
    np.testing.assert_allclose(post, O.posterior(t, obs, off), rtol=RTOL, atol=1e-300)


def test_reference_layer_api(gpu):
    """optimizer.py-shaped wrappers: types and block-order summation."""
    g = golden("sweep_syn27.npz")
    a, b, pi, obs, off = g["a"], g["b"], g["pi"], g["obs"], g["off"]
    V_lst = [obs[off[k]:off[k + 1]].astype(np.int64) for k in range(len(off) - 1)]
    acc = 0
    for v in g["loglik"].tolist():
        acc += v
    tot = hmm.loglik_wrapper(a, b, pi, V_lst)
    assert isinstance(tot, float)
    assert abs(tot - acc) <= 1e-10 * abs(acc)
    paths = hmm.viterbi_wrapper(a, b, pi, V_lst)
    assert all(p.dtype == np.float64 for p in paths)
    np.testing.assert_array_equal(np.concatenate(paths), g["path"].astype(np.float64))
    posts = hmm.post_prob_wrapper(a, b, pi, V_lst)
    assert [p.shape for p in posts] == [(len(v), a.shape[0]) for v in V_lst]
    assert abs(hmm.forward_loglik(a, b, pi, V_lst[2]) - g["loglik"][2]) <= 1e-10 * abs(acc)
    with pytest.raises(IndexError):
        hmm.loglik_wrapper(a, b, pi, [np.array([0, 625])])


def test_device_layer_matches_host_layer(gpu):
    import torch

    g = golden("sweep_syn70.npz")
    model, plan = hmm.Model(g["a"], g["b"], g["pi"]), hmm.Plan(g["off"])
    d_obs = torch.from_numpy(g["obs"].astype(np.int16)).to(gpu)
    ll = hmm.forward_loglik_device(model, plan, d_obs).cpu().numpy()
    path = hmm.viterbi_device(model, plan, d_obs).cpu().numpy()
    post = hmm.posterior_device(model, plan, d_obs).cpu().numpy()
    torch.cuda.synchronize()
    np.testing.assert_array_equal(ll, hmm.block_logliks(model, plan, g["obs"]))
    np.testing.assert_array_equal(path, g["path"])
    np.testing.assert_array_equal(post, hmm._posteriors(model, plan, g["obs"]))
    assert hmm.last_kernel_ms("viterbi") > 0


@pytest.mark.parametrize("n", [5, 65, 70, 72, 133, 192])
def test_viterbi_frequent_switches(gpu, n):
    """Weakly sticky transitions and sharp emissions: the path switches every few columns,
    so nearly every 16-column tile holds several clear stay flags and the traceback rebuilds
    omega rows from the tile checkpoint and reuses them for later switches in the tile."""
    rng = np.random.default_rng(40 + n)
    a, b, pi = random_hmm(rng, n, stay=(0.2, 0.6))
    b = rng.dirichlet(np.full(256, 0.05), size=n)
    lengths = [1, 2, 15, 16, 17, 31, 32, 33, 1023, 1024, 1025, 3000] + \
        list(rng.integers(1, 700, size=20))
    obs, off, _ = sample_alignment(a, b, pi, lengths, seed=n, p_n=0.01, p_gap=0.01)
    t = build_tables(a, b, pi)
    ref = O.viterbi(t, obs, off)
    assert (np.diff(ref.astype(np.int64)) != 0).mean() > 0.1  # the regime under test
    model, plan = hmm.Model(a, b, pi), hmm.Plan(off)
    np.testing.assert_array_equal(hmm._paths(model, plan, obs), ref)


@pytest.mark.parametrize("n", [46, 65, 70, 72])
def test_forward_viterbi_call_matches_separate_calls(gpu, n):
    """itr_forward_viterbi (forward sweep beside the Viterbi sweep's longest blocks on a
    disjoint CU set) returns what itr_forward_loglik and itr_viterbi return (paths bit for
    bit, log-likelihoods to 1e-12), and both match the oracle.  Blocks of 2,048+ columns go to
    the long-block launch; blocks of half the longest or more are split forward tasks."""
    import torch

    rng = np.random.default_rng(70 + n)
    a, b, pi = random_hmm(rng, n)
    lengths = [9000, 7000, 6000, 4000, 3000, 2500] + list(rng.integers(1, 1500, size=300))
    obs, off, _ = sample_alignment(a, b, pi, lengths, seed=n, p_n=0.02, p_gap=0.02)
    t = build_tables(a, b, pi)
    model, plan = hmm.Model(a, b, pi), hmm.Plan(off)
    d_obs = torch.from_numpy(obs.astype(np.int16)).to(gpu)
    ll1 = hmm.forward_loglik_device(model, plan, d_obs).cpu().numpy()
    p1 = hmm.viterbi_device(model, plan, d_obs).cpu().numpy()
    ll2, p2 = hmm.forward_viterbi_device(model, plan, d_obs)
    ll2, p2 = ll2.cpu().numpy(), p2.cpu().numpy()
    # the combined call's forward may use another layout (per-wave FMA chains): the same
    # log-likelihoods to rounding, the same paths bit for bit
    np.testing.assert_allclose(ll2, ll1, rtol=1e-12, atol=0)
    np.testing.assert_array_equal(p2, p1)
    np.testing.assert_array_equal(p2, O.viterbi(t, obs, off))
    np.testing.assert_allclose(ll2, O.forward_loglik(t, obs, off), rtol=RTOL, atol=0)


@pytest.mark.parametrize("n", [46, 70, 133])
def test_few_long_blocks_forward_viterbi(gpu, n):
    """The few-block branch of itr_forward_viterbi (capi.cpp viterbi_impl `few`: no more
    blocks than 3/4 of the CUs and no per-wave layout, e.g. 100 x 100 kbp): the Viterbi sweep
    on a masked set of CUs, one per block, the forward on the others at the same time.  96
    equally long blocks of 5,000 columns (every block in the long set, so the partition's
    long work exceeds half the chip and the per-wave layout is off at n = 70 too): the
    combined call against the separate calls (paths bit for bit, log-likelihoods 1e-12) and
    against the oracle."""
    import torch

    rng = np.random.default_rng(90 + n)
    a, b, pi = random_hmm(rng, n)
    lengths = [5000] * 96
    obs, off, _ = sample_alignment(a, b, pi, lengths, seed=n, p_n=0.02, p_gap=0.02)
    t = build_tables(a, b, pi)
    model, plan = hmm.Model(a, b, pi), hmm.Plan(off)
    d_obs = torch.from_numpy(obs.astype(np.int16)).to(gpu)
    ll1 = hmm.forward_loglik_device(model, plan, d_obs).cpu().numpy()
    p1 = hmm.viterbi_device(model, plan, d_obs).cpu().numpy()
    ll2, p2 = hmm.forward_viterbi_device(model, plan, d_obs)
    ll2, p2 = ll2.cpu().numpy(), p2.cpu().numpy()
    np.testing.assert_allclose(ll2, ll1, rtol=1e-12, atol=0)
    np.testing.assert_array_equal(p2, p1)
    np.testing.assert_array_equal(p2, O.viterbi(t, obs, off))
    np.testing.assert_allclose(ll2, O.forward_loglik(t, obs, off), rtol=RTOL, atol=0)


def test_wrappers_host_blocks_paths(gpu):
    """loglik_wrapper / viterbi_wrapper on int64 blocks (the pinned host-block entry points,
    itr_forward_loglik_blocks / itr_viterbi_blocks) against the same calls on int32 blocks
    (the NumPy packing path) and the goldens: identical results; a symbol outside the
    alphabet raises IndexError naming its block and column; a model or layout change after a
    cached call is a new cache entry."""
    g = golden("sweep_syn70.npz")
    a, b, pi, obs, off = g["a"], g["b"], g["pi"], g["obs"], g["off"]
    V64 = [obs[off[k]:off[k + 1]].astype(np.int64) for k in range(len(off) - 1)]
    V32 = [v.astype(np.int32) for v in V64]
    for _ in range(2):  # second round: cached model and plan
        assert hmm.loglik_wrapper(a, b, pi, V64) == hmm.loglik_wrapper(a, b, pi, V32)
        p64, p32 = hmm.viterbi_wrapper(a, b, pi, V64), hmm.viterbi_wrapper(a, b, pi, V32)
        assert all(x.dtype == np.float64 for x in p64)
        np.testing.assert_array_equal(np.concatenate(p64), np.concatenate(p32))
        np.testing.assert_array_equal(np.concatenate(p64), g["path"].astype(np.float64))
    W = [v.copy() for v in V64]
    W[2][7] = 625
    with pytest.raises(IndexError, match="block 2, column 7"):
        hmm.loglik_wrapper(a, b, pi, W)
    with pytest.raises(IndexError, match="block 2, column 7"):
        hmm.viterbi_wrapper(a, b, pi, W)
    # another model with the same layout, and the same model on a sub-layout
    a2 = np.ascontiguousarray(a[::-1, ::-1])
    b2, pi2 = np.ascontiguousarray(b[::-1]), np.ascontiguousarray(pi[::-1])
    t2 = build_tables(a2, b2, pi2)
    np.testing.assert_array_equal(np.concatenate(hmm.viterbi_wrapper(a2, b2, pi2, V64)),
                                  O.viterbi(t2, obs, off).astype(np.float64))
    sub = V64[1:3]
    so = np.concatenate(sub).astype(np.uint16)
    soff = np.concatenate([[0], np.cumsum([len(v) for v in sub])])
    ll = hmm.loglik_wrapper(a, b, pi, sub)
    ref = O.forward_loglik(build_tables(a, b, pi), so, soff)
    assert abs(ll - (ref[0] + ref[1])) <= 1e-9 * abs(ll)


@pytest.mark.parametrize("n", [133, 141, 144])
def test_single_long_block_vs_oracle(gpu, n):
    """One block only: the forward sweep has no matrix-core group (every task is a VALU
    half of the split block), the Viterbi runs the lane-group layout alone, and at
    N = 137..144 both must cover every source state (sources 136..143 were outside the
    previous VALU configurations' lanes)."""
    rng = np.random.default_rng(77 + n)
    a, b, pi = random_hmm(rng, n)
    obs, off, _ = sample_alignment(a, b, pi, [5000], seed=n, p_n=0.03, p_gap=0.02)
    t = build_tables(a, b, pi)
    ll, path, post = run_all(a, b, pi, obs, off)
    np.testing.assert_allclose(ll, O.forward_loglik(t, obs, off), rtol=RTOL, atol=0)
    np.testing.assert_array_equal(path, O.viterbi(t, obs, off))
    np.testing.assert_allclose(post, O.posterior(t, obs, off), rtol=RTOL, atol=1e-300)
