"""Host-side pieces of the model build (CPU): state spaces, cutpoints, coalescence
integrals, and the whole chain/emission bookkeeping on a NumPy stand-in backend
(tests/helpers/np_linalg.py) against the reference's golden model."""
import numpy as np
import pytest
from scipy import integrate, stats

from conftest import golden

from itrails_amd.model.emissions import (cutpoints_AB, cutpoints_ABC, double_table,
                                         single_table)
from itrails_amd.model.statespace import omega_nonrev_counts, omega_of_key, state_space


def test_state_space_sizes_and_rates():
    for s, n, nt in ((1, 2, 2), (2, 15, 44), (3, 203, 1118)):
        ss = state_space(s)
        assert ss.n == n and len(ss.transitions) == nt
        Q = ss.rate_matrix(1.3, 0.7)
        assert np.allclose(Q.sum(1), 0.0, atol=1e-12)
        assert sum(m.sum() for m in ss.omega_masks.values()) == n
    assert omega_nonrev_counts(3) == {0: 0, 3: 1, 5: 1, 6: 1, 7: 2}
    assert omega_of_key(((-1, -1, -1), (0, 1, -1))) == (0, 3)
    assert omega_of_key(((-1, 2, 2), (3, 1, 4))) == (7, 7)


def test_cutpoints_match_scipy():
    for n, tab, c in ((1, 0.8, 1.0), (3, 0.8, 1.0), (5, 0.3, 1.7)):
        ref = stats.truncexpon.ppf(np.arange(n + 1) / n, b=tab * c, scale=1 / c)
        assert np.array_equal(cutpoints_AB(n, tab, c), ref)
        ref = stats.expon.ppf(np.arange(n + 1) / n, scale=1 / c)
        assert np.array_equal(cutpoints_ABC(n, c), ref)


def _P(x, y, tau, mu):
    return 0.25 + ((1.0 if x == y else 0.0) - 0.25) * np.exp(-mu * tau)


def test_single_coalescence_table_by_quadrature():
    t, mu, k = 0.9, 0.4, 1.3
    F = single_table(t, mu, k)
    for a, b, c in ((0, 0, 0), (0, 1, 2), (3, 3, 1)):
        f = lambda s: sum(k * np.exp(-k * s) / (1 - np.exp(-k * t)) * _P(a, d, s, mu) *
                          _P(d, b, s, mu) * _P(d, c, t - s, mu) for d in range(4))
        assert abs(F[a, b, c] - integrate.quad(f, 0, t, epsabs=1e-15)[0]) < 1e-13


def test_double_coalescence_table_by_quadrature():
    t, mu = 0.8, 0.3
    DD = double_table(t, mu)
    den = 1 + 0.5 * np.exp(-3 * t) - 1.5 * np.exp(-t)
    for a, b, c, d in ((0, 0, 0, 0), (0, 1, 2, 3)):
        g = lambda s2, s1: sum(3 * np.exp(-3 * s1) * np.exp(-(s2 - s1)) * _P(a, e, s1, mu) *
                               _P(e, b, s1, mu) * _P(e, f, s2 - s1, mu) * _P(f, c, s2, mu) *
                               _P(f, d, t - s2, mu) / den for e in range(4) for f in range(4))
        v = integrate.dblquad(g, 0, t, lambda s1: s1, lambda s1: t, epsabs=1e-14)[0]
        assert abs(DD[a, b, c, d] - v) < 1e-12


@pytest.mark.parametrize("name", ["model_kat_1_1.npz"])
def test_model_bookkeeping_on_host_backend(name):
    from helpers.np_linalg import NumpyLinalg
    from itrails_amd.model import trans_emiss_calc
    g = golden(name)
    n_ab, n_abc = (int(x) for x in g["n_int"])
    a, b, pi, hidden, _ = trans_emiss_calc(*g["args"], n_ab, n_abc, la=NumpyLinalg())
    assert np.array_equal(np.array([hidden[i] for i in range(len(hidden))]), g["hidden"])
    assert np.allclose(a, g["a"], rtol=1e-10, atol=1e-15)
    assert np.allclose(pi, g["pi"], rtol=1e-10, atol=1e-15)
    assert np.allclose(b, g["b"], rtol=1e-8, atol=1e-15)


@pytest.mark.parametrize("name", ["model_kat_3_3.npz"])
def test_device_chain_routes_like_host_chain(name):
    """The device-resident planned chain (torch tensors) and the host planned chain (NumPy)
    fed the same deterministic stand-in matrix functions give the same model: every row,
    group sum, overwrite and closing contraction is routed identically (helpers/torch_linalg)."""
    from helpers.torch_linalg import FakeNumpyLinalg, FakeTorchLinalg
    from itrails_amd.model import trans_emiss_calc
    g = golden(name)
    n_ab, n_abc = (int(x) for x in g["n_int"])
    la_h, la_d = FakeNumpyLinalg(), FakeTorchLinalg()
    a_h, _, pi_h, _, _ = trans_emiss_calc(*g["args"], n_ab, n_abc, la=la_h)
    a_d, _, pi_d, _, _ = trans_emiss_calc(*g["args"], n_ab, n_abc, la=la_d)
    assert la_d.stats["vanloan"] > la_h.stats["vanloan"] > 0  # + the propagator jobs
    assert np.allclose(a_d, a_h, rtol=1e-12, atol=0) and np.allclose(pi_d, pi_h, rtol=1e-12)


def test_coalescence_tables_vs_reference_closed_forms():
    """single_table / double_table against the reference's own closed forms summed in its
    order (tests/golden/coal_tables.npz: p_b_c_given_a_JC69_analytical and
    p_b_c_d_given_a_JC69_analytical, get_emission_prob_mat.py:95-118, 400-424) at the KAT
    model's (t, mu) and one larger mu.  Entries of order (mu t)^3 come out of a cancellation
    of O(1) terms in both closed forms (at mu = 4/3000 both lose up to ~1e-4 of such an entry
    against a 30-digit quadrature), so the bar is the table's scale: |x - ref| <= 4e-15 max
    |ref|, and 1e-12 relative where nothing cancels (mu = 0.3)."""
    g = golden("coal_tables.npz")
    for (t, mu, k), S, D in zip(g["cases"], g["single"], g["double"]):
        s, d = single_table(t, mu, k), double_table(t, mu)
        assert np.abs(s - S).max() <= 4e-15 * np.abs(S).max()
        assert np.abs(d - D).max() <= 4e-15 * np.abs(D).max()
        if mu > 0.1:
            np.testing.assert_allclose(s, S, rtol=1e-12, atol=0)
            np.testing.assert_allclose(d, D, rtol=1e-12, atol=0)


def test_closed_form_propagators_vs_expm():
    """The host's closed forms of the build's small exponentials against scipy's expm: the
    JC69-form branch generators (emissions.jc69_propagators) and the one-species two-state
    chains (chains._expm2), within a few ulp of the matrix scale."""
    import scipy.linalg as sl
    from itrails_amd.model.chains import _expm2
    from itrails_amd.model.emissions import generator_matrices, jc69_propagators
    from itrails_amd.model.statespace import state_space
    rng = np.random.default_rng(3)
    gens = [(a, -3.0 * a) for a in rng.random(50) * 2.0] + [(0.0, 0.0), (0.3, -0.7)]
    P = jc69_propagators(gens)
    for g, m in zip(gens, generator_matrices(gens)):
        ref = sl.expm(m)
        assert np.abs(P[gens.index(g)] - ref).max() <= 5e-14 * np.abs(ref).max()
    for coal, rho, t in [(0.7, 0.3, 0.5), (1.2, 1e-3, 3.0), (1.0, 2.0, 1e-4), (0.0, 0.0, 1.0)]:
        Q = state_space(1).rate_matrix(coal, rho)
        ref = sl.expm(Q * t)
        assert np.abs(_expm2(Q, t) - ref).max() <= 5e-14 * np.abs(ref).max()
