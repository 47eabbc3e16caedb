"""Batched dense FP64 linear algebra on the GPU (itrails_amd/csrc/dense.hip) behind the
reference's own call surface.

* `expm(A)` — the reference's `expm` (expm.py:9-167): same Pade branch per 1-norm, same
  scaling and squaring; returns a NumPy array.  `expm_batched` runs any number of matrices
  of one order in one call (the model build batches every distinct propagator of a
  rebuild).
* `solve_batched`, `gemm_batched` — device LU solve / MFMA GEMM for the Van Loan and
  deepest-interval contractions.

Inputs may be NumPy arrays (copied to the current device and back) or torch.cuda float64
tensors (used in place; results stay on the device).  No host fallback: without the
library or a device every call raises.
"""
from __future__ import annotations

import numpy as np

from ._lib import check, lib

__all__ = ["expm", "expm_batched", "expm_blocktri_batched", "vanloan_paths", "vanloan_job_norms",
           "solve_batched", "inverse_batched", "gemm_batched"]


_PINNED: dict = {}  # shape -> ring of [pinned host tensor, event of its last copy]
_RING = 4


def h2d(x):
    """A float64 host array on the current device without a host-side wait: the copy goes
    through a pinned staging buffer (a ring of four per shape, each reused only after its
    previous copy is done).  A copy from pageable memory would wait for every kernel queued
    before it on the stream, so each one in the model build stalled the host until the
    device was idle."""
    import torch
    a = np.ascontiguousarray(x, dtype=np.float64)
    ring = _PINNED.get(a.shape)
    if ring is None:
        if len(_PINNED) > 64:
            _PINNED.clear()
        ring = _PINNED[a.shape] = [0, [[torch.empty(a.shape, dtype=torch.float64,
                                                    pin_memory=True), None]
                                       for _ in range(_RING)]]
    slot = ring[1][ring[0]]
    ring[0] = (ring[0] + 1) % _RING
    if slot[1] is not None:
        slot[1].synchronize()
    slot[0].numpy()[...] = a
    out = slot[0].to("cuda", non_blocking=True)
    ev = torch.cuda.Event()
    ev.record()
    slot[1] = ev
    return out


def _dev(x):
    import torch
    if isinstance(x, torch.Tensor):
        if not x.is_cuda or x.dtype != torch.float64:
            raise TypeError("expected a torch.cuda float64 tensor")
        return x.contiguous(), True
    return h2d(x), False


def _stream():
    import torch
    return torch.cuda.current_stream().cuda_stream


def expm_batched(A):
    """expm of every A[b] (shape (B, n, n)); NumPy in -> NumPy out, CUDA tensor in -> out."""
    import torch
    d, on_dev = _dev(A)
    if d.dim() != 3 or d.shape[1] != d.shape[2]:
        raise ValueError("expected a (batch, n, n) array")
    out = torch.empty_like(d)
    if d.shape[0]:
        check(lib().itr_expm_batched(d.shape[1], d.shape[0], d.data_ptr(), out.data_ptr(),
                                     _stream()))
    return out if on_dev else out.cpu().numpy()


def expm_blocktri_batched(A, n_blocks: int):
    """expm of every A[b] whose n_blocks x n_blocks block structure is upper triangular with
    equal diagonal blocks (Van Loan matrices, vanloan.py:392-425): same result as
    expm_batched, only the upper blocks are formed (lower blocks of the result are zero)."""
    import torch
    d, on_dev = _dev(A)
    if d.dim() != 3 or d.shape[1] != d.shape[2] or d.shape[1] % n_blocks:
        raise ValueError("expected a (batch, k*n, k*n) array")
    out = torch.empty_like(d)
    if d.shape[0]:
        check(lib().itr_expm_blocktri_batched(d.shape[1] // n_blocks, n_blocks, d.shape[0],
                                              d.data_ptr(), out.data_ptr(), _stream()))
    return out if on_dev else out.cpu().numpy()


def _vanloan_args(Q, t, masks_u8, path_job, path_off, path_mask):
    Q = np.ascontiguousarray(Q, dtype=np.float64)
    t = np.ascontiguousarray(t, dtype=np.float64)
    masks_u8 = np.ascontiguousarray(masks_u8, dtype=np.uint8)
    path_job = np.ascontiguousarray(path_job, dtype=np.int32)
    path_off = np.ascontiguousarray(path_off, dtype=np.int64)
    path_mask = np.ascontiguousarray(path_mask, dtype=np.int32)
    n = Q.shape[0]
    if Q.ndim != 2 or Q.shape[1] != n or masks_u8.ndim != 2 or \
            (masks_u8.size and masks_u8.shape[1] != n):
        raise ValueError("expected Q (n, n) and masks (n_masks, n)")
    if len(path_off) != len(path_job) + 1:
        raise ValueError("path_off must have n_paths + 1 entries")
    return Q, t, masks_u8, path_job, path_off, path_mask


def vanloan_paths(Q, t, masks_u8, path_job, path_off, path_mask, job_norm=None):
    """Van Loan integrals of many omega paths in one shared evaluation (itr_vanloan_paths):
    returns a torch.cuda (n_paths, n, n) tensor, entry p = expm(C_p t[path_job[p]])[:n, -n:]
    with C_p the block bidiagonal matrix of vanloan.py:392-425 for the mask ids
    path_mask[path_off[p]:path_off[p+1]] (a length-1 path gives expm(Q t)).  Q, t, masks and
    the path arrays are host NumPy arrays; nothing is synchronised.  `job_norm` (per
    interval, from vanloan_job_norms of a superset of the paths) fixes each interval's Pade
    branch and scaling to that superset's (itr_vanloan_paths_ex)."""
    import torch
    Q, t, masks_u8, path_job, path_off, path_mask = _vanloan_args(
        Q, t, masks_u8, path_job, path_off, path_mask)
    n = Q.shape[0]
    npaths = len(path_job)
    out = torch.empty((npaths, n, n), dtype=torch.float64, device="cuda")
    if npaths:
        jn = None
        if job_norm is not None:
            jn = np.ascontiguousarray(job_norm, dtype=np.float64)
            if jn.shape != (len(t),):
                raise ValueError("job_norm must have one entry per interval")
        check(lib().itr_vanloan_paths_ex(n, Q.ctypes.data, len(t), t.ctypes.data,
                                         masks_u8.shape[0], masks_u8.ctypes.data, npaths,
                                         path_job.ctypes.data, path_off.ctypes.data,
                                         path_mask.ctypes.data,
                                         jn.ctypes.data if jn is not None else None,
                                         out.data_ptr(), _stream()))
    return out


def vanloan_job_norms(Q, t, masks_u8, path_job, path_off, path_mask):
    """Per interval, the largest ||C_p t||_1 of its paths (itr_vanloan_job_norms, host
    only): the input of expm.py:16-143's Pade branch choice."""
    Q, t, masks_u8, path_job, path_off, path_mask = _vanloan_args(
        Q, t, masks_u8, path_job, path_off, path_mask)
    out = np.zeros(len(t), dtype=np.float64)
    check(lib().itr_vanloan_job_norms(Q.shape[0], Q.ctypes.data, len(t), t.ctypes.data,
                                      masks_u8.shape[0], masks_u8.ctypes.data, len(path_job),
                                      path_job.ctypes.data, path_off.ctypes.data,
                                      path_mask.ctypes.data, out.ctypes.data))
    return out


def expm(A):
    """Matrix exponential of one square matrix (expm.py:9).  The reference divides its
    argument in place by 2**s on the Pade-13 branch (expm.py:141-143); every reference call
    site passes a temporary, so the argument is left untouched here."""
    A = np.asarray(A, dtype=np.float64)
    if A.ndim != 2 or A.shape[0] != A.shape[1]:
        raise ValueError("expm expects a square matrix")
    return expm_batched(A[None])[0]


def solve_batched(M, R):
    """X with M[b] X[b] = R[b] (LU with partial pivoting); M (B,n,n), R (B,n,k)."""
    import torch
    dM, on_dev = _dev(M)
    dR, _ = _dev(R)
    dM = dM.clone()
    dR = dR.clone()
    if dM.dim() != 3 or dR.dim() != 3 or dM.shape[1] != dM.shape[2] or \
            dR.shape[:2] != dM.shape[:2]:
        raise ValueError("expected M (batch, n, n) and R (batch, n, k)")
    if dM.shape[0]:
        check(lib().itr_solve_batched(dM.shape[1], dR.shape[2], dM.shape[0], dM.data_ptr(),
                                      dR.data_ptr(), _stream()))
    return dR if on_dev else dR.cpu().numpy()


def inverse_batched(M):
    """M[b]^-1 for every b (itr_inverse_batched: Gauss-Jordan in registers for n <= 208)."""
    import torch
    dM, on_dev = _dev(M)
    if dM.dim() != 3 or dM.shape[1] != dM.shape[2]:
        raise ValueError("expected M (batch, n, n)")
    dM = dM.contiguous()
    out = torch.empty_like(dM)
    if dM.shape[0]:
        check(lib().itr_inverse_batched(dM.shape[1], dM.shape[0], dM.data_ptr(), out.data_ptr(),
                                        _stream()))
    return out if on_dev else out.cpu().numpy()


def gemm_batched(A, B, alpha=1.0):
    """alpha * A[b] @ B[b] for every b."""
    import torch
    dA, on_dev = _dev(A)
    dB, _ = _dev(B)
    if dA.dim() != 3 or dB.dim() != 3 or dA.shape[0] != dB.shape[0] or dA.shape[2] != dB.shape[1]:
        raise ValueError("shape mismatch")
    C = torch.empty((dA.shape[0], dA.shape[1], dB.shape[2]), dtype=torch.float64,
                    device=dA.device)
    if dA.shape[0]:
        check(lib().itr_gemm_batched(dA.shape[1], dB.shape[2], dA.shape[2], dA.shape[0],
                                     float(alpha), dA.data_ptr(), dB.data_ptr(), 0.0,
                                     C.data_ptr(), _stream()))
    return C if on_dev else C.cpu().numpy()


def chain_rows(P, F, M, tab, out, cols=None):
    """One interval's chain-step products on device (itr_chain_rows): for the entries of
    `tab` = (src, oms, ome, dst, ngroups, rmax) (int32 device tensors [ngroups * rmax], -1
    padding; oms / ome may be None), out[dst] = ((P[src][:, cols] * F[oms]) @ M[g]) * F[ome]."""
    src, oms, ome, dst, ng, rmax = tab
    k = M.shape[-1]
    p = lambda x: x.data_ptr() if x is not None else None  # noqa: E731
    check(lib().itr_chain_rows(k, ng, rmax, p(src), p(oms), p(ome), p(dst), p(cols), P.data_ptr(),
                               P.shape[1], p(F), F.shape[1] if F is not None else 0,
                               M.data_ptr(), out.data_ptr(), out.shape[1], _stream()))
    return out


def group_sum(S, off, paths, ng, out=None):
    """M[g] = S[paths[off[g]]] + S[paths[off[g] + 1]] + ... in path order (itr_group_sum);
    off / paths: int32 device tensors."""
    import torch
    nn = S[0].numel() if S.shape[0] else int(np.prod(S.shape[1:]))
    if out is None:
        out = torch.empty((ng,) + tuple(S.shape[1:]), dtype=torch.float64, device=S.device)
    if ng:
        check(lib().itr_group_sum(nn, ng, off.data_ptr(), paths.data_ptr(),
                                  S.data_ptr() if S.numel() else None, out.data_ptr(), _stream()))
    return out
