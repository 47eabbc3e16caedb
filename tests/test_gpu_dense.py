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


@pytest.mark.parametrize("n,batch,dominant", [(1, 3, True), (2, 2, False), (7, 3, False),
                                              (31, 2, True), (33, 3, False), (64, 2, False),
                                              (201, 2, True), (203, 3, False), (208, 2, True),
                                              (208, 1, False), (230, 2, False)])
def test_inverse_matches_lapack(gpu, n, batch, dominant):
    """itr_inverse_batched against LAPACK's inverse: diagonally dominant matrices take the
    pass without interchanges, general ones (and one dominant member beside them) the
    pivoting pass; n = 230 the blocked-LU fallback."""
    from itrails_amd.dense import inverse_batched
    rng = np.random.default_rng(n * 7 + batch)
    M = rng.standard_normal((batch, n, n))
    if dominant:
        M += np.eye(n) * (np.abs(M).sum(axis=1, keepdims=True) + 1.0)
    elif batch > 1:
        M[0] += np.eye(n) * (np.abs(M[0]).sum(axis=0) + 1.0)  # a pass-1 member in the batch
    X = inverse_batched(M)
    ref = np.linalg.inv(M)
    for b in range(batch):
        err = np.abs(X[b] - ref[b]).max() / np.abs(ref[b]).max()
        assert err < 1e-11 * max(1.0, np.linalg.cond(M[b]) / 1e3), (n, b, err)


def test_inverse_pivoting_pattern(gpu):
    """A zero leading pivot and interchanges at several steps (the pivoting pass's row and
    column interchanges), and the model build's matrix shape: a rate matrix of order 201."""
    from itrails_amd.dense import inverse_batched
    M = np.array([[[0.0, 1.0, 2.0], [3.0, 4.0, 5.0], [6.0, 7.0, 9.0]]])
    assert np.allclose(inverse_batched(M)[0], np.linalg.inv(M[0]), rtol=1e-12, atol=1e-12)
    rng = np.random.default_rng(5)
    P = np.eye(64)[rng.permutation(64)]
    A = P @ (np.eye(64) * 10 + rng.standard_normal((64, 64)))  # rows shuffled: swaps needed
    assert np.allclose(inverse_batched(A[None])[0], np.linalg.inv(A), rtol=1e-10, atol=1e-12)
    Q = rng.random((201, 201)) * (rng.random((201, 201)) < 0.05)
    np.fill_diagonal(Q, 0.0)
    np.fill_diagonal(Q, -Q.sum(axis=1) - rng.random(201) * 0.1)
    ref = np.linalg.inv(Q)
    assert np.allclose(inverse_batched(Q[None])[0], ref, rtol=1e-11, atol=1e-13 * np.abs(ref).max())


@pytest.mark.parametrize("m,n,k", [(1, 1, 1), (1, 203, 203), (203, 203, 203), (70, 17, 129),
                                   (64, 64, 16), (65, 63, 17)])
def test_gemm_matches_blas(gpu, m, n, k):
    from itrails_amd.dense import gemm_batched
    rng = np.random.default_rng(m + 7 * n + 13 * k)
    A = rng.standard_normal((3, m, k))
    B = rng.standard_normal((3, k, n))
    C = gemm_batched(A, B, alpha=-2.0)
    assert np.allclose(C, -2.0 * A @ B, rtol=1e-12, atol=1e-12 * k)


def _vanloan_like(rng, n, k, scale):
    """Block upper bidiagonal k x k blocks: a rate matrix Q (rows sum to 0) on the diagonal,
    masked copies of Q above it (vanloan.py:392-425), times `scale`."""
    Q = rng.random((n, n)) * (rng.random((n, n)) < 0.2)
    np.fill_diagonal(Q, 0.0)
    np.fill_diagonal(Q, -Q.sum(axis=1))
    C = np.zeros((n * k, n * k))
    for b in range(k):
        C[b * n:(b + 1) * n, b * n:(b + 1) * n] = Q
    for b in range(1, k):
        m0, m1 = rng.random(n) < 0.5, rng.random(n) < 0.5
        C[(b - 1) * n:b * n, b * n:(b + 1) * n] = m0[:, None] * Q * m1[None, :]
    return C * scale


@pytest.mark.parametrize("n,k", [(5, 2), (17, 3), (40, 4), (64, 5), (70, 2)])
def test_expm_blocktri_matches_dense(gpu, n, k):
    """Block-triangular Van Loan expm (only the upper blocks formed, back substitution
    through the diagonal block) against the dense batched expm and scipy, every Pade branch
    (norms from 1e-3 to 30)."""
    import scipy.linalg as sl
    from itrails_amd.dense import expm_batched, expm_blocktri_batched
    rng = np.random.default_rng(n * 10 + k)
    A = np.stack([_vanloan_like(rng, n, k, s) for s in (1e-3, 0.05, 0.3, 0.7, 1.5, 4.0, 30.0)])
    B = expm_blocktri_batched(A, k)
    D = expm_batched(A)
    for b in range(A.shape[0]):
        ref = sl.expm(A[b])
        for i in range(k):
            for j in range(k):
                blk = np.s_[i * n:(i + 1) * n, j * n:(j + 1) * n]
                if i > j:
                    assert not B[b][blk].any()
                    continue
                scale = max(np.abs(ref[blk]).max(), 1e-300)
                assert np.abs(B[b][blk] - D[b][blk]).max() <= 1e-12 * max(scale, 1.0)
                assert np.abs(B[b][blk] - ref[blk]).max() <= 1e-11 * max(scale, 1.0)


@pytest.mark.parametrize("n,nmask", [(5, 3), (17, 4), (70, 6), (203, 9)])
def test_vanloan_paths_shared_matches_per_path(gpu, n, nmask):
    """itr_vanloan_paths (shared sub-path evaluation, one Pade branch and scaling per
    interval) against scipy's expm of each path's block matrix: paths of length 1..5 that
    share prefixes and suffixes, three intervals whose norms select different branches and
    squaring counts, duplicates and interleaved intervals in the request order."""
    import scipy.linalg as sl
    from itrails_amd.dense import vanloan_paths
    rng = np.random.default_rng(n + 1000 * nmask)
    Q = rng.random((n, n)) * (rng.random((n, n)) < 0.3)
    np.fill_diagonal(Q, 0.0)
    np.fill_diagonal(Q, -Q.sum(axis=1))
    Q /= max(1.0, np.abs(Q).sum(axis=0).max())  # ||Q||_1 <= 1
    masks = (rng.random((nmask, n)) < 0.5).astype(np.uint8)
    t = np.array([0.02, 0.6, 9.0])  # Pade 5-7, 9-13 without / with squarings
    paths = []
    for _ in range(40):
        L = int(rng.integers(1, 6))
        paths.append((int(rng.integers(0, 3)), [int(x) for x in rng.integers(0, nmask, L)]))
    paths += [paths[3], (paths[5][0], paths[5][1][:2]), (2, [0]), (0, [1, 2, 1, 2, 1])]
    job = np.array([j for j, _ in paths], dtype=np.int32)
    off = np.zeros(len(paths) + 1, dtype=np.int64)
    np.cumsum([len(p) for _, p in paths], out=off[1:])
    pm = np.array([w for _, p in paths for w in p], dtype=np.int32)
    got = vanloan_paths(Q, t, masks, job, off, pm).cpu().numpy()
    for k, (j, p) in enumerate(paths):
        L = len(p)
        C = np.zeros((n * L, n * L))
        for b in range(L):
            C[b * n:(b + 1) * n, b * n:(b + 1) * n] = Q
        for b in range(1, L):
            C[(b - 1) * n:b * n, b * n:(b + 1) * n] = masks[p[b - 1]][:, None] * Q * \
                masks[p[b]][None, :]
        ref = sl.expm(C * t[j])[:n, -n:]
        scale = max(np.abs(ref).max(), 1e-300)
        assert np.abs(got[k] - ref).max() <= 1e-11 * max(scale, 1.0), (k, j, L)


@pytest.mark.parametrize("n,ncls", [(40, 5), (203, 16)])
def test_vanloan_paths_compact_supports(gpu, n, ncls):
    """The support-compressed evaluation on a nearly acyclic CTMC like the coalescent ones:
    states in ordered classes, transitions only within a class or to later classes, masks
    = classes.  Non-root members then live on small rectangles (rows reaching the first
    class, columns reached from the last); the result matches scipy's expm of every path's
    block matrix, including the exact zeros outside the rectangle.  A subset of the paths
    evaluated with the norms of the whole set (the rank-split build) gives the same matrices
    bit for bit."""
    import scipy.linalg as sl
    from itrails_amd.dense import vanloan_job_norms, vanloan_paths
    rng = np.random.default_rng(7 * n + ncls)
    cls = np.sort(rng.integers(0, ncls, n))
    Q = rng.random((n, n)) * (rng.random((n, n)) < 0.25)
    Q *= cls[None, :] >= cls[:, None]  # no transition back to an earlier class
    np.fill_diagonal(Q, 0.0)
    np.fill_diagonal(Q, -Q.sum(axis=1))
    Q /= max(1.0, np.abs(Q).sum(axis=0).max())
    masks = np.stack([(cls == c).astype(np.uint8) for c in range(ncls)])
    t = np.array([0.3, 2.5, 40.0])
    paths = []
    for _ in range(60):
        L = int(rng.integers(1, 6))
        seq = np.sort(rng.choice(ncls, L, replace=L > ncls))
        paths.append((int(rng.integers(0, 3)), [int(x) for x in seq]))
    job = np.array([j for j, _ in paths], dtype=np.int32)
    off = np.zeros(len(paths) + 1, dtype=np.int64)
    np.cumsum([len(p) for _, p in paths], out=off[1:])
    pm = np.array([w for _, p in paths for w in p], dtype=np.int32)
    got = vanloan_paths(Q, t, masks, job, off, pm).cpu().numpy()
    for k, (j, p) in enumerate(paths):
        L = len(p)
        C = np.zeros((n * L, n * L))
        for b in range(L):
            C[b * n:(b + 1) * n, b * n:(b + 1) * n] = Q
        for b in range(1, L):
            C[(b - 1) * n:b * n, b * n:(b + 1) * n] = masks[p[b - 1]][:, None] * Q * \
                masks[p[b]][None, :]
        ref = sl.expm(C * t[j])[:n, -n:]
        scale = max(np.abs(ref).max(), 1e-300)
        assert np.abs(got[k] - ref).max() <= 1e-11 * max(scale, 1.0), (k, j, L)
        assert not got[k][ref == 0.0].any(), (k, "non-zero outside the support")
    # a subset with the whole set's norms: same branch, bit-identical matrices
    norms = vanloan_job_norms(Q, t, masks, job, off, pm)
    sel = np.arange(0, len(paths), 3)
    soff = np.zeros(len(sel) + 1, dtype=np.int64)
    np.cumsum([len(paths[i][1]) for i in sel], out=soff[1:])
    spm = np.array([w for i in sel for w in paths[i][1]], dtype=np.int32)
    sub = vanloan_paths(Q, t, masks, job[sel], soff, spm, job_norm=norms).cpu().numpy()
    assert np.array_equal(sub, got[sel])


def test_vanloan_paths_interval_branch_vs_per_path(gpu):
    """One Pade branch and scaling per interval (itr_vanloan_paths: chosen from the largest
    ||C_p t||_1 of the interval's paths) against the reference's per-path choice
    (expm.py:9-167, here the device's per-matrix branch selection in expm_blocktri_batched):
    paths of length 1 and 5 with empty and full masks in ONE interval, whose norms straddle
    the Pade-9 / Pade-13 threshold (theta_9 = 2.10), so the short paths get a higher degree
    and more squarings than the reference would give them.  The results agree to rounding
    (1e-13 of the block's scale), which is the deviation DESIGN.md §4 states."""
    from itrails_amd.dense import expm_blocktri_batched, vanloan_paths
    rng = np.random.default_rng(4242)
    n = 40
    Q = rng.random((n, n)) * (rng.random((n, n)) < 0.3)
    np.fill_diagonal(Q, 0.0)
    np.fill_diagonal(Q, -Q.sum(axis=1))
    Q /= np.abs(Q).sum(axis=0).max()  # ||Q||_1 = 1
    masks = np.stack([np.zeros(n), np.ones(n), (rng.random(n) < 0.5)]).astype(np.uint8)
    t = np.array([1.2])  # ||Q t|| = 1.2 < theta_9; five full-mask blocks: ~3 > theta_9
    paths = [[0], [1], [0, 0, 0, 0, 0], [1, 1, 1, 1, 1], [2, 1, 2], [0, 2, 1, 1, 0]]
    job = np.zeros(len(paths), dtype=np.int32)
    off = np.zeros(len(paths) + 1, dtype=np.int64)
    np.cumsum([len(p) for p in paths], out=off[1:])
    pm = np.array([w for p in paths for w in p], dtype=np.int32)
    got = vanloan_paths(Q, t, masks, job, off, pm).cpu().numpy()
    for k, p in enumerate(paths):
        L = len(p)
        C = np.zeros((n * L, n * L))
        for b in range(L):
            C[b * n:(b + 1) * n, b * n:(b + 1) * n] = Q
        for b in range(1, L):
            C[(b - 1) * n:b * n, b * n:(b + 1) * n] = masks[p[b - 1]][:, None] * Q * \
                masks[p[b]][None, :]
        ref = expm_blocktri_batched((C * t[0])[None], L)[0][:n, -n:]
        scale = max(np.abs(ref).max(), 1.0)
        assert np.abs(got[k] - ref).max() <= 1e-13 * scale, (k, np.abs(got[k] - ref).max())


@pytest.mark.parametrize("k,ng,rmax", [(203, 3, 70), (15, 1, 5), (130, 2, 200)])
def test_chain_rows_vs_numpy(gpu, k, ng, rmax):
    """itr_chain_rows (the fused chain-step products of the device model build) against the
    same gathers, masks and products in NumPy: every written row, padding rows untouched."""
    import torch
    from itrails_amd.dense import chain_rows

    rng = np.random.default_rng(k + ng)
    n = k + 7 if k == 130 else k  # (column gather: P wider than the matrices)
    nrows = ng * rmax + 5
    P = rng.random((nrows, n))
    F = (rng.random((9, k)) < 0.7).astype(np.float64)
    M = rng.random((ng, k, k)) / k
    src = rng.integers(0, nrows, size=ng * rmax).astype(np.int32)
    src[rng.random(src.size) < 0.2] = -1
    oms = rng.integers(0, 9, size=src.size).astype(np.int32)
    ome = rng.integers(0, 9, size=src.size).astype(np.int32)
    dst = rng.permutation(nrows)[:src.size].astype(np.int32)
    cols = np.sort(rng.choice(n, size=k, replace=False)).astype(np.int32) if n > k else None
    d = lambda x: torch.from_numpy(x).to(gpu) if x is not None else None  # noqa: E731
    out = torch.full((nrows, k), -1.0, dtype=torch.float64, device=gpu)
    use_masks = cols is None
    tab = (d(src), d(oms) if use_masks else None, d(ome) if use_masks else None, d(dst), ng, rmax)
    chain_rows(d(P), d(F) if use_masks else None, d(M), tab, out, cols=d(cols))
    got = out.cpu().numpy()
    want = np.full((nrows, k), -1.0)
    for e in range(src.size):
        if src[e] < 0:
            continue
        v = P[src[e]][cols] if cols is not None else P[src[e]].copy()
        if use_masks:
            v = v * F[oms[e]]
        r = v @ M[e // rmax]
        want[dst[e]] = r * F[ome[e]] if use_masks else r
    np.testing.assert_allclose(got, want, rtol=1e-12, atol=1e-15)
