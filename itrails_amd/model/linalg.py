"""Batched propagators of the model build on the GPU.

Every matrix function the reference evaluates one call at a time — `expm` of interval
propagators (get_joint_prob_mat.py:119-123, run_markov_chain_AB.py:135,
run_markov_chain_ABC.py:347), Van Loan block exponentials (vanloan.py:392-425) and
deepest-interval inverses (deepest_ti.py:215-256) — is requested here as a list, de-duplicated,
assembled on the device and evaluated as one batch by the HIP kernels of dense.hip
(itr_expm_batched / itr_solve_batched).
"""
from __future__ import annotations

from contextlib import contextmanager
from typing import Dict, List, Sequence, Tuple

import numpy as np

Omega = Tuple[int, int]

_SPLIT_GROUP = [None]  # process group of a rank-split model build, see split_build
_DP_CACHE: Dict = {}  # deepest_t index tensors per (device, paths), see _deepest_plan


@contextmanager
def split_build(enabled: bool = True, group=None):
    """Model builds started inside this context on a torch.distributed job divide their
    de-duplicated Van Loan work across the ranks of `group` (run_markov_chain_ABC.py:118-195
    fans the reference's tasks out over processes the same way): the three-species chain's
    propagators and path groups are cut into runs of equal Van Loan cost, one run per rank
    (chains.split_partition), each rank forming its groups' sums; one all-gather gives every
    rank all intervals' propagators and group matrices, bit-identical to a one-rank build.
    Every rank of the group must build the same model at the same time (the optimizer's
    objective evaluations do)."""
    prev = _SPLIT_GROUP[0]
    _SPLIT_GROUP[0] = ("on", group) if enabled else None
    try:
        yield
    finally:
        _SPLIT_GROUP[0] = prev


class DeviceLinalg:
    """The product backend: torch.cuda for memory, dense.hip for the arithmetic."""

    def __init__(self):
        import torch
        if not torch.cuda.is_available():
            raise RuntimeError("the model build needs an MI355X (no host fallback)")
        self.torch = torch
        self.dev = torch.device("cuda", torch.cuda.current_device())
        self.stats = {"expm": 0, "vanloan": 0, "deepest": 0}
        self.rank, self.world, self.group = 0, 1, None
        if _SPLIT_GROUP[0] is not None:
            import torch.distributed as dist
            if dist.is_available() and dist.is_initialized():
                self.group = _SPLIT_GROUP[0][1]
                self.rank = dist.get_rank(self.group)
                self.world = dist.get_world_size(self.group)

    def expm(self, mats: Sequence[np.ndarray]) -> List[np.ndarray]:
        from ..dense import expm_batched
        if not len(mats):
            return []
        by_n: Dict[int, List[int]] = {}
        for i, m in enumerate(mats):
            by_n.setdefault(m.shape[0], []).append(i)
        out: List[np.ndarray] = [None] * len(mats)
        for n, idx in by_n.items():
            A = np.stack([np.asarray(mats[i], dtype=np.float64) for i in idx])
            E = expm_batched(A)
            for k, i in enumerate(idx):
                out[i] = E[k]
        self.stats["expm"] += len(mats)
        return out

    def _block_matrices(self, Q, masks, paths, L, scale, diag_blocks):
        """(G, n*b, n*b) device tensor: `diag_blocks` diagonal blocks Q*scale and, between
        consecutive classes p[i-1] -> p[i], the super-diagonal block
        diag(mask p[i-1]) Q diag(mask p[i]) * scale (vanloan.py:415-423,
        deepest_ti.py:236-250)."""
        torch = self.torch
        n = Q.shape[0]
        b = diag_blocks
        dQ = torch.from_numpy(Q).to(self.dev)
        G = len(paths)
        C = torch.zeros((G, n * b, n * b), dtype=torch.float64, device=self.dev)
        Qs = dQ * scale if scale is not None else dQ
        for blk in range(b):
            C[:, blk * n:(blk + 1) * n, blk * n:(blk + 1) * n] = Qs
        for blk in range(1, b):
            ma = torch.from_numpy(np.stack([masks[p[blk - 1]] for p in paths]).astype(np.float64)).to(self.dev)
            mb = torch.from_numpy(np.stack([masks[p[blk]] for p in paths]).astype(np.float64)).to(self.dev)
            A = ma[:, :, None] * dQ[None] * mb[:, None, :]
            if scale is not None:
                A = A * scale
            C[:, (blk - 1) * n:blk * n, blk * n:(blk + 1) * n] = A
        return C

    # ---- device-resident forms (torch.cuda tensors out; used by the planned chains) -----
    def vanloan_batch(self, Q: np.ndarray, masks_u8: np.ndarray, t: np.ndarray,
                      path_job: np.ndarray, path_off: np.ndarray, path_mask: np.ndarray,
                      job_norm=None):
        """(n_paths, n, n) device tensor of Van Loan integrals over several intervals at once
        (dense.vanloan_paths: shared sub-path evaluation, vanloan.hip); `job_norm` fixes the
        intervals' Pade branches (vanloan_norms of a superset of the paths)."""
        from ..dense import vanloan_paths
        self.stats["vanloan"] += len(path_job)
        return vanloan_paths(Q, t, masks_u8, path_job, path_off, path_mask, job_norm)

    def vanloan_norms(self, Q: np.ndarray, masks_u8: np.ndarray, t: np.ndarray,
                      path_job: np.ndarray, path_off: np.ndarray, path_mask: np.ndarray):
        """Per interval, the largest ||C_p t||_1 of its paths (host only)."""
        from ..dense import vanloan_job_norms
        return vanloan_job_norms(Q, t, masks_u8, path_job, path_off, path_mask)

    def deepest_t(self, Q: np.ndarray, masks: Dict[Omega, np.ndarray],
                  paths: Sequence[Tuple[Omega, ...]]):
        """(n_paths, n, n) device tensor of the deepest-interval integrals (deepest_ti.py:
        215-256): (-C^-1)[:n, -n:] @ A_{L-1} for the block upper bidiagonal C of path p
        (diagonal blocks Q, super-diagonal A_i = diag(m p[i-1]) Q diag(m p[i])).  The top-right
        block of the inverse of such a matrix is (-1)^(L-2) Q^-1 A_1 Q^-1 ... A_{L-2} Q^-1, so
        the integral is (-1)^(L-1) G_1 G_2 ... G_{L-1} with G_i = Q^-1 A_i: one inverse of
        Q, one batched GEMM for every distinct omega pair, then the chain products per path
        length (MFMA GEMMs, dense.hip) — instead of one LU of order (L-1) n per path."""
        from ..dense import gemm_batched, h2d, inverse_batched
        torch = self.torch
        n = Q.shape[0]
        out = torch.empty((len(paths), n, n), dtype=torch.float64, device=self.dev)
        if not len(paths):
            return out
        plan = self._deepest_plan(masks, paths, n)
        dQ = h2d(Q)
        Qinv = inverse_batched(dQ[None])[0]
        A = (plan["ma"][:, :, None] * dQ[None] * plan["mb"][:, None, :]).contiguous()
        G = gemm_batched(Qinv.expand(A.shape[0], n, n).contiguous(), A)
        for L, idx, cols in plan["by_len"]:
            R = G[cols[0]]
            for k in range(1, L - 1):
                R = gemm_batched(R.contiguous(), G[cols[k]].contiguous())
            out[idx] = R if (L - 1) % 2 == 0 else -R
        self.stats["deepest"] += len(paths)
        return out

    def _deepest_plan(self, masks, paths, n):
        """deepest_t's index tensors for one list of paths (the same every rebuild): the
        distinct omega pairs' mask rows and, per path length, the pair ids of each step."""
        torch = self.torch
        key = (str(self.dev), n, tuple(tuple(p) for p in paths), tuple(masks))
        cache = _DP_CACHE
        plan = cache.get(key)
        if plan is not None:
            return plan
        pair_id: Dict = {}
        for p in paths:
            for i in range(1, len(p)):
                pair_id.setdefault((p[i - 1], p[i]), len(pair_id))
        pl = list(pair_id)
        dev = self.dev
        ma = torch.from_numpy(np.stack([masks[a] for a, _ in pl]).astype(np.float64)).to(dev)
        mb = torch.from_numpy(np.stack([masks[b] for _, b in pl]).astype(np.float64)).to(dev)
        by_len: Dict[int, List[int]] = {}
        for i, p in enumerate(paths):
            by_len.setdefault(len(p), []).append(i)
        steps = []
        for L, idx in sorted(by_len.items()):
            gi = np.asarray([[pair_id[(paths[i][k - 1], paths[i][k])] for k in range(1, L)]
                             for i in idx], dtype=np.int64)
            steps.append((L, torch.as_tensor(idx, device=dev),
                          [torch.from_numpy(np.ascontiguousarray(gi[:, k])).to(dev)
                           for k in range(L - 1)]))
        plan = {"ma": ma, "mb": mb, "by_len": steps}
        if len(cache) > 8:
            cache.clear()
        cache[key] = plan
        return plan

    # ---- host-array forms (the dictionary chains, the introgression model) ---------------
    def vanloan(self, Q: np.ndarray, t: float, masks: Dict[Omega, np.ndarray],
                paths: Sequence[Tuple[Omega, ...]]) -> List[np.ndarray]:
        """expm(C t)[:n, -n:] for each omega path (vanloan.py:392-425), one shared
        evaluation of all paths (vanloan.hip)."""
        if not len(paths):
            return []
        keys = list(masks)
        mid = {k: i for i, k in enumerate(keys)}
        mu8 = np.stack([np.asarray(masks[k], dtype=np.uint8) for k in keys])
        off = np.zeros(len(paths) + 1, dtype=np.int64)
        np.cumsum([len(p) for p in paths], out=off[1:])
        pm = np.asarray([mid[w] for p in paths for w in p], dtype=np.int32)
        S = self.vanloan_batch(Q, mu8, np.asarray([t], dtype=np.float64),
                               np.zeros(len(paths), dtype=np.int32), off, pm).cpu().numpy()
        return list(S)

    def deepest(self, Q: np.ndarray, masks: Dict[Omega, np.ndarray],
                paths: Sequence[Tuple[Omega, ...]]) -> List[np.ndarray]:
        """deepest_t as host arrays."""
        if not len(paths):
            return []
        return list(self.deepest_t(Q, masks, paths).cpu().numpy())

    def chain_rows(self, P, F, M, tab, out, cols=None):
        """One interval's chain-step products, gathered, masked and scattered in one fused
        MFMA pass (dense.chain_rows, itr_chain_rows)."""
        from ..dense import chain_rows
        return chain_rows(P, F, M, tab, out, cols=cols)

    def rowmat(self, V: np.ndarray, M: np.ndarray) -> np.ndarray:
        """V @ M for a stack of row vectors V (k x n) and one n x n propagator: the per-key
        vector-matrix products of a chain interval as one MFMA GEMM (dense.hip)."""
        from ..dense import gemm_batched
        if V.shape[0] == 0:
            return np.zeros((0, M.shape[1]))
        return gemm_batched(np.ascontiguousarray(V)[None], np.ascontiguousarray(M)[None])[0]

    def emission_rows(self, tables: np.ndarray) -> np.ndarray:
        """Emission rows of every state from its packed tables (emission.hip)."""
        from .._lib import check, lib
        torch = self.torch
        from ..dense import h2d
        dt = h2d(tables)
        out = torch.empty((tables.shape[0], 256), dtype=torch.float64, device=self.dev)
        check(lib().itr_emission_rows(tables.shape[0], dt.data_ptr(), out.data_ptr(),
                                      torch.cuda.current_stream().cuda_stream))
        return out.cpu().numpy()
