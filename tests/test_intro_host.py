"""Introgression model build on the host: the generated CTMC state
spaces against load_trans_mat's CSV chains (int_load_trans_mat.py:6-41) and the
hand-written missing-lineage chain (int_get_joint_prob_mat.py:306-339), and the model
bookkeeping against the reference's trans_emiss_calc_introgression output
(tests/golden/model_int_*.npz) on the NumPy test backend."""
import json
import os
from ast import literal_eval

import numpy as np
import pytest

from itrails_amd.model import intro

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def _space():
    with open(os.path.join(GOLDEN, "int_statespace.json")) as f:
        return json.load(f)


def _name(st):
    return repr([tuple(b) for b in st])


@pytest.mark.parametrize("n_seq,masks", [(1, [1]), (2, [1, 2]), (3, [1, 2, 4])])
def test_chain_matches_reference_csv(n_seq, masks):
    ref = _space()[str(n_seq)]
    states = intro.one_seq(1) if n_seq == 1 else intro.chain_states(masks)
    assert len(states) == ref["n_states"]
    sym = intro.symbols(states)
    got = sorted([_name(states[i]), _name(states[j]), str(sym[i, j])]
                 for i in range(len(states)) for j in range(len(states)) if sym[i, j] != "0")
    assert got == ref["transitions"]
    # positional conventions the reference relies on
    if n_seq == 1:
        assert [_name(s) for s in states] == ref["first"]
    if n_seq == 3:
        assert [_name(s) for s in states[-2:]] == ref["absorbing_last_two"]


def test_missing_lineage_chain():
    ref = _space()["miss"]
    assert [_name(s) for s in intro.MISS_BC] == ref["states"]
    sym = intro.symbols(intro.MISS_BC)
    assert [[str(v) for v in row] for row in sym] == ref["symbols"]


def test_rate_matrix_rows_sum_to_zero():
    q = intro.rate_matrix(intro.symbols(intro.chain_states([1, 2, 4])), 1.3, 0.7)
    assert q.shape == (203, 203)
    assert np.allclose(q.sum(axis=1), 0, atol=1e-12)
    assert set(np.unique(q[~np.eye(203, dtype=bool)])) <= {0.0, 1.3, 0.7}


def test_task_lists_cover_every_state_pair():
    # the reference's case lists enumerate every (l, L, r, R) / (L, r, R) combination
    n = 4
    assert len(intro._pool_abc_list(n)) == n * (n + 1) * (n * n + n + 2) // 8
    assert len(intro._pool_ab_list(n)) == n * n * (n + 1) // 2


@pytest.mark.parametrize("name", ["model_int_ikat_1_1.npz"])
def test_intro_model_bookkeeping_on_host_backend(name):
    from helpers.np_linalg import NumpyLinalg
    g = np.load(os.path.join(GOLDEN, name))
    n_ab, n_abc = (int(x) for x in g["n_int"])
    a, b, pi, hidden, observed = intro.trans_emiss_calc_introgression(
        *g["args"], n_ab, n_abc, la=NumpyLinalg())
    assert np.array_equal(np.array([hidden[i] for i in range(len(hidden))]), g["hidden"])
    assert [observed[i] for i in range(256)] == list(g["observed"])
    assert np.allclose(a, g["a"], rtol=1e-10, atol=1e-15)
    assert np.allclose(pi, g["pi"], rtol=1e-10, atol=1e-15)
    assert np.allclose(b, g["b"], rtol=1e-8, atol=1e-15)
