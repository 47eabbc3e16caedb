"""Batched propagators of the model build on the GPU.

Every matrix function the reference evaluates one call at a time — `expm` of interval
propagators (get_joint_prob_mat.py:119-123, run_markov_chain_AB.py:135,
run_markov_chain_ABC.py:347), Van Loan block exponentials (vanloan.py:392-425) and
deepest-interval inverses (deepest_ti.py:215-256) — is requested here as a list, de-duplicated,
assembled on the device and evaluated as one batch by the HIP kernels of dense.hip
(itr_expm_batched / itr_solve_batched).
"""
from __future__ import annotations

from typing import Dict, List, Sequence, Tuple

import numpy as np

Omega = Tuple[int, int]


class DeviceLinalg:
    """The product backend: torch.cuda for memory, dense.hip for the arithmetic."""

    def __init__(self):
        import torch
        if not torch.cuda.is_available():
            raise RuntimeError("the model build needs an MI355X (no host fallback)")
        self.torch = torch
        self.dev = torch.device("cuda", torch.cuda.current_device())
        self.stats = {"expm": 0, "vanloan": 0, "deepest": 0}

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
                      path_job: np.ndarray, path_off: np.ndarray, path_mask: np.ndarray):
        """(n_paths, n, n) device tensor of Van Loan integrals over several intervals at once
        (dense.vanloan_paths: shared sub-path evaluation, vanloan.hip)."""
        from ..dense import vanloan_paths
        self.stats["vanloan"] += len(path_job)
        return vanloan_paths(Q, t, masks_u8, path_job, path_off, path_mask)

    def deepest_t(self, Q: np.ndarray, masks: Dict[Omega, np.ndarray],
                  paths: Sequence[Tuple[Omega, ...]]):
        """(n_paths, n, n) device tensor: (-C^-1)[:n, -n:] @ (diag(m p[-2]) Q diag(m p[-1]))
        for each omega path (deepest_ti.py:215-256); the last n columns of C^-1 come from one
        batched solve against the last n columns of the identity, per path length."""
        from ..dense import gemm_batched, solve_batched
        torch = self.torch
        n = Q.shape[0]
        out = torch.empty((len(paths), n, n), dtype=torch.float64, device=self.dev)
        by_len: Dict[int, List[int]] = {}
        for i, p in enumerate(paths):
            by_len.setdefault(len(p), []).append(i)
        dQ = torch.from_numpy(Q).to(self.dev)
        for L, idx in sorted(by_len.items()):
            steps = L - 1
            sub = [paths[i] for i in idx]
            C = self._block_matrices(Q, masks, sub, steps, None, steps)
            G = len(sub)
            R = torch.zeros((G, n * steps, n), dtype=torch.float64, device=self.dev)
            R[:, (steps - 1) * n:, :] = torch.eye(n, dtype=torch.float64, device=self.dev)
            X = solve_batched(C, R)[:, :n, :]
            ma = torch.from_numpy(np.stack([masks[p[-2]] for p in sub]).astype(np.float64)).to(self.dev)
            mb = torch.from_numpy(np.stack([masks[p[-1]] for p in sub]).astype(np.float64)).to(self.dev)
            A = (ma[:, :, None] * dQ[None] * mb[:, None, :]).contiguous()
            out[torch.as_tensor(idx, device=self.dev)] = gemm_batched(X.contiguous(), A,
                                                                      alpha=-1.0)
        self.stats["deepest"] += len(paths)
        return out

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
        dt = torch.from_numpy(np.ascontiguousarray(tables, dtype=np.float64)).to(self.dev)
        out = torch.empty((tables.shape[0], 256), dtype=torch.float64, device=self.dev)
        check(lib().itr_emission_rows(tables.shape[0], dt.data_ptr(), out.data_ptr(),
                                      torch.cuda.current_stream().cuda_stream))
        return out.cpu().numpy()
