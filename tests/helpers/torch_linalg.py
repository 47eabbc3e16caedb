"""Stand-ins for checking the device-resident form of the planned three-species chain
(chains._run_chain_abc_device: one Van Loan batch for all intervals, key rows as one tensor,
group sums in path order, padded batched row products, closing contractions) on the CPU —
TEST INFRASTRUCTURE ONLY.

The two fakes return the same deterministic pseudo-random matrices for every Van Loan /
deepest-interval request (seeded by the path's mask rows and the interval length), one as
NumPy lists for the host form (_run_chain_abc_planned), one as torch CPU tensors for the
device form.  Equal chain outputs then show that the device form routes every row, group,
sum and overwrite exactly like the host form; the matrix functions themselves are checked on
the GPU against the reference's models."""
import hashlib

import numpy as np
import torch

from helpers.np_linalg import NumpyLinalg


def _fake(n, rows, t):
    h = hashlib.sha256(b"".join(r.tobytes() for r in rows) + np.float64(t).tobytes())
    rng = np.random.default_rng(int.from_bytes(h.digest()[:8], "little"))
    return rng.random((n, n)) * 1e-2


def _fake_q(Qt):
    """Stand-in for expm(Q t) (a length-1 path or an interval propagator), seeded by the
    matrix Q t itself so both requests get the same matrix."""
    return _fake(Qt.shape[0], [np.ascontiguousarray(Qt)], 0.0)


class FakeNumpyLinalg(NumpyLinalg):
    def vanloan(self, Q, t, masks, paths):
        self.stats["vanloan"] += len(paths)
        n = Q.shape[0]
        return [_fake(n, [np.asarray(masks[w], dtype=np.uint8) for w in p], t) if len(p) > 1
                else _fake_q(Q * t) for p in paths]

    def deepest(self, Q, masks, paths):
        self.stats["deepest"] += len(paths)
        n = Q.shape[0]
        return [_fake(n, [np.asarray(masks[w], dtype=np.uint8) for w in p], -1.0)
                for p in paths]

    def expm(self, mats):  # interval propagators: a length-1 "path"
        self.stats["expm"] += len(mats)
        return [_fake_q(m) if m.shape[0] > 100 else super(FakeNumpyLinalg, self).expm([m])[0]
                for m in mats]


class FakeTorchLinalg(FakeNumpyLinalg):
    dev = torch.device("cpu")
    rank, world, group = 0, 1, None

    def vanloan_batch(self, Q, masks_u8, t, path_job, path_off, path_mask, job_norm=None):
        n = Q.shape[0]
        out = []
        for p in range(len(path_job)):
            ids = path_mask[path_off[p]:path_off[p + 1]]
            j = int(path_job[p])
            out.append(_fake(n, [np.asarray(masks_u8[i], dtype=np.uint8) for i in ids], t[j])
                       if len(ids) > 1 else _fake_q(Q * t[j]))
        self.stats["vanloan"] += len(path_job)
        return torch.from_numpy(np.stack(out)) if out else torch.zeros((0, n, n),
                                                                       dtype=torch.float64)

    def vanloan_norms(self, Q, masks_u8, t, path_job, path_off, path_mask):
        return np.zeros(len(t))

    def deepest_t(self, Q, masks, paths):
        n = Q.shape[0]
        D = self.deepest(Q, masks, paths)
        return torch.from_numpy(np.stack(D)) if D else torch.zeros((0, n, n),
                                                                   dtype=torch.float64)

    def chain_rows(self, P, F, M, tab, out, cols=None):
        """The semantics of itr_chain_rows in torch (CPU)."""
        src, oms, ome, dst, ng, rmax = tab
        for e in range(ng * rmax):
            s = int(src[e])
            if s < 0:
                continue
            v = P[s][cols.long()] if cols is not None else P[s]
            if oms is not None:
                v = v * F[int(oms[e])]
            # (np.einsum: one fixed summation order whatever the thread count, so the split
            # build's ranks and the single-rank build round alike)
            Mg = M[e // rmax] if M.dim() == 3 else M
            r = torch.from_numpy(np.einsum("i,ij->j", v.numpy(), Mg.numpy()))
            if ome is not None:
                r = r * F[int(ome[e])]
            out[int(dst[e])] = r
        return out
