"""The CPU oracle (oracle/hmm_oracle.c) pinned against the reference's own outputs.

tests/golden/sweep_*.npz hold forward_loglik / viterbi+backtrack / post_prob results the
reference produced (tests/golden/make_golden.py).  The oracle is the checker for the device
sweeps, so it must reproduce them first: loglik to 1e-12 relative, Viterbi paths exactly.
"""
import numpy as np
import pytest

from conftest import golden, sweep_fixtures
from itrails_amd.tables import build_tables
from oracle import hmm_oracle as O


@pytest.mark.parametrize("name", sweep_fixtures())
def test_oracle_vs_reference(name):
    g = golden(name)
    t = build_tables(g["a"], g["b"], g["pi"])
    ll = O.forward_loglik(t, g["obs"], g["off"])
    np.testing.assert_allclose(ll, g["loglik"], rtol=1e-12, atol=0)
    path = O.viterbi(t, g["obs"], g["off"])
    np.testing.assert_array_equal(path, g["path"])
    post = O.posterior(t, g["obs"], g["off"])
    np.testing.assert_allclose(post[g["post_rows"]], g["post"], rtol=1e-9, atol=1e-300)


def test_fixture_paths_switch_states():
    # a backtracking bug is invisible on paths that never leave one state; the
    # reference's own models barely switch, so the synthetic fixtures carry this check
    for name in [f for f in sweep_fixtures() if f.startswith("sweep_syn")]:
        g = golden(name)
        assert (np.diff(g["path"]) != 0).sum() > 5, name


@pytest.mark.parametrize("name", ["sweep_syn4.npz", "sweep_syn13.npz", "sweep_kat_3_3.npz"])
def test_rows_oracle_vs_reference(name):
    """The row-level restatement (oracle/rows_oracle.py, the checker of itr_block_rows)
    reproduces the reference's own outputs: log-likelihood from log alpha, the path from
    (omega, prev), posterior rows from log alpha + log beta."""
    from oracle import rows_oracle as R

    g = golden(name)
    t = build_tables(g["a"], g["b"], g["pi"])
    obs, off = g["obs"].astype(np.int64), g["off"]
    for k in range(len(off) - 1):
        V = obs[off[k]:off[k + 1]]
        if V.size == 0:
            continue
        alpha = R.forward(t, V)
        assert abs(R.loglik_from_alpha(alpha) - g["loglik"][k]) <= 1e-8 * abs(g["loglik"][k])
        om, prev = R.viterbi(t, V)
        np.testing.assert_array_equal(R.backtrack_viterbi(om, prev), g["path"][off[k]:off[k + 1]])
        post = R.post_from_rows(alpha, R.backward(t, V))
        rows = g["post_rows"]
        sel = (rows >= off[k]) & (rows < off[k + 1])
        np.testing.assert_allclose(post[rows[sel] - off[k]], g["post"][sel], rtol=1e-8, atol=1e-300)
