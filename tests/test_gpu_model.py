"""Model build on the GPU (itrails_amd.model.trans_emiss_calc on DeviceLinalg: batched expm /
Van Loan / deepest-interval solves / emission contraction in HIP) against the reference's
own trans_emiss_calc outputs (tests/golden/model_*.npz, SURVEY 8c KAT and an asymmetric
parameter set)."""
import time

import numpy as np
import pytest

from conftest import golden, int_model_fixtures, model_fixtures

pytestmark = pytest.mark.gpu

# a and pi: products/sums of propagators, agree to ~1e-15; b: the closed-form coalescence
# integrals are evaluated by a different (term-wise exact) expansion, small entries agree to
# ~1e-9 relative
A_RTOL, B_RTOL, ATOL = 1e-10, 1e-8, 1e-15


@pytest.mark.parametrize("name", [m for m in model_fixtures()])
def test_trans_emiss_calc_matches_reference(gpu, name):
    from itrails_amd.model import trans_emiss_calc
    from itrails_amd.model.linalg import DeviceLinalg
    g = golden(name)
    n_ab, n_abc = (int(x) for x in g["n_int"])
    la = DeviceLinalg()
    t0 = time.time()
    a, b, pi, hidden, observed = trans_emiss_calc(*g["args"], n_ab, n_abc, la=la)
    dt = time.time() - t0
    hid = np.array([hidden[i] for i in range(len(hidden))])
    assert (hid == g["hidden"]).all()
    assert [observed[i] for i in range(256)] == list(g["observed"])
    assert np.allclose(a, g["a"], rtol=A_RTOL, atol=ATOL), np.abs(a - g["a"]).max()
    assert np.allclose(pi, g["pi"], rtol=A_RTOL, atol=ATOL)
    assert np.allclose(b, g["b"], rtol=B_RTOL, atol=ATOL), np.abs(b - g["b"]).max()
    print(f"{name}: N={a.shape[0]} built in {dt:.2f}s (reference {float(g['build_seconds']):.1f}s)"
          f" stats={la.stats}")


@pytest.mark.parametrize("name", [m for m in int_model_fixtures()])
def test_trans_emiss_calc_introgression_matches_reference(gpu, name):
    """The introgression model (int_get_trans_emiss.py:9-185) against the reference's own
    output; the reference evaluates its propagators with scipy.linalg.expm, the device with
    the itrails Pade branches (dense.hip), so a/pi agree to rounding, not bit for bit."""
    from itrails_amd.model.intro import trans_emiss_calc_introgression
    from itrails_amd.model.linalg import DeviceLinalg
    g = golden(name)
    n_ab, n_abc = (int(x) for x in g["n_int"])
    la = DeviceLinalg()
    t0 = time.time()
    a, b, pi, hidden, observed = trans_emiss_calc_introgression(*g["args"], n_ab, n_abc, la=la)
    dt = time.time() - t0
    hid = np.array([hidden[i] for i in range(len(hidden))])
    assert (hid == g["hidden"]).all()
    assert [observed[i] for i in range(256)] == list(g["observed"])
    assert np.allclose(a, g["a"], rtol=A_RTOL, atol=ATOL), np.abs(a - g["a"]).max()
    assert np.allclose(pi, g["pi"], rtol=A_RTOL, atol=ATOL)
    assert np.allclose(b, g["b"], rtol=B_RTOL, atol=ATOL), np.abs(b - g["b"]).max()
    print(f"{name}: N={a.shape[0]} built in {dt:.2f}s (reference {float(g['build_seconds']):.1f}s)"
          f" stats={la.stats}")
