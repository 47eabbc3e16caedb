"""Batched expm / solve / GEMM on the GPU (itrails_amd/csrc/dense.hip) against the golden
vectors of the reference's expm (tests/golden/expm_kat.npz: expm.py:9-167 on rate matrices
whose 1-norms straddle every Pade branch threshold and several squaring counts) and against
NumPy's LAPACK/BLAS for solve and GEMM."""
import numpy as np
import pytest

from conftest import golden

pytestmark = pytest.mark.gpu

# expm tolerance: entries are probabilities/propagators; the GPU sums in a different order
# than BLAS/LAPACK, so entries agree to ~1e-14 relative to the matrix scale
RTOL, ATOL_SCALE = 1e-10, 1e-13


def _close(x, y):
    scale = max(1.0, float(np.abs(y).max()))
    return np.allclose(x, y, rtol=RTOL, atol=ATOL_SCALE * scale)


@pytest.mark.parametrize("n", [2, 4, 15, 31, 203])
def test_expm_matches_reference_golden(gpu, n):
    from itrails_amd.dense import expm_batched, expm
    g = golden("expm_kat.npz")
    A, E = g[f"A_{n}"], g[f"E_{n}"]
    got = expm_batched(A)
    for b in range(len(A)):
        assert _close(got[b], E[b]), (n, b, np.abs(got[b] - E[b]).max())
    assert _close(expm(A[0]), E[0])


def test_expm_mixed_branches_one_batch(gpu):
    """Members of one batch take different Pade branches and squaring counts."""
    from itrails_amd.dense import expm_batched
    g = golden("expm_kat.npz")
    A = np.concatenate([g["A_15"], g["A_15"][::-1]])
    E = np.concatenate([g["E_15"], g["E_15"][::-1]])
    got = expm_batched(A)
    for b in range(len(A)):
        assert _close(got[b], E[b])


@pytest.mark.parametrize("n,k,batch", [(1, 1, 3), (5, 2, 4), (33, 7, 3), (64, 64, 2),
                                       (203, 203, 2), (406, 203, 1)])
def test_solve_matches_lapack(gpu, n, k, batch):
    from itrails_amd.dense import solve_batched
    rng = np.random.default_rng(n * 131 + k)
    M = rng.standard_normal((batch, n, n)) + n * np.eye(n) * rng.random((batch, 1, 1))
    R = rng.standard_normal((batch, n, k))
    X = solve_batched(M, R)
    ref = np.linalg.solve(M, R)
    assert np.allclose(X, ref, rtol=1e-9, atol=1e-11 * np.abs(ref).max())


def test_solve_needs_pivoting(gpu):
    from itrails_amd.dense import solve_batched
    M = np.array([[[0.0, 1.0, 2.0], [3.0, 4.0, 5.0], [6.0, 7.0, 9.0]]])
    R = np.eye(3)[None]
    assert np.allclose(solve_batched(M, R)[0], np.linalg.inv(M[0]), rtol=1e-12, atol=1e-12)


@pytest.mark.parametrize("m,n,k", [(1, 1, 1), (1, 203, 203), (203, 203, 203), (70, 17, 129),
                                   (64, 64, 16), (65, 63, 17)])
def test_gemm_matches_blas(gpu, m, n, k):
    from itrails_amd.dense import gemm_batched
    rng = np.random.default_rng(m + 7 * n + 13 * k)
    A = rng.standard_normal((3, m, k))
    B = rng.standard_normal((3, k, n))
    C = gemm_batched(A, B, alpha=-2.0)
    assert np.allclose(C, -2.0 * A @ B, rtol=1e-12, atol=1e-12 * k)
