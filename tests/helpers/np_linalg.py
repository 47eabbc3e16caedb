"""Host (NumPy/SciPy) stand-in for itrails_amd.model.linalg.DeviceLinalg — TEST
INFRASTRUCTURE ONLY.  It lets the CPU test-suite check the model-build bookkeeping (state
spaces, chain branching, path enumeration, emission tables) against the reference's
golden models without a GPU; the GPU tests run the same code on DeviceLinalg."""
import numpy as np
import scipy.linalg as sl


class NumpyLinalg:
    def __init__(self):
        self.stats = {"expm": 0, "vanloan": 0, "deepest": 0}

    def expm(self, mats):
        self.stats["expm"] += len(mats)
        return [sl.expm(np.asarray(m, dtype=np.float64)) for m in mats]

    @staticmethod
    def _block(Q, masks, p, b, scale):
        n = Q.shape[0]
        C = np.zeros((n * b, n * b))
        Qs = Q * scale if scale is not None else Q
        for k in range(b):
            C[k * n:(k + 1) * n, k * n:(k + 1) * n] = Qs
        for k in range(1, b):
            A = masks[p[k - 1]][:, None] * Q * masks[p[k]][None, :]
            C[(k - 1) * n:k * n, k * n:(k + 1) * n] = A * scale if scale is not None else A
        return C

    def vanloan(self, Q, t, masks, paths):
        self.stats["vanloan"] += len(paths)
        n = Q.shape[0]
        return [sl.expm(self._block(Q, masks, p, len(p), t))[:n, -n:] for p in paths]

    def deepest(self, Q, masks, paths):
        self.stats["deepest"] += len(paths)
        n = Q.shape[0]
        out = []
        for p in paths:
            C = self._block(Q, masks, p, len(p) - 1, None)
            A = masks[p[-2]][:, None] * Q * masks[p[-1]][None, :]
            out.append((-np.linalg.inv(C))[:n, -n:] @ A)
        return out

    def rowmat(self, V, M):
        return V @ M

    def emission_rows(self, tab):
        out = np.zeros((tab.shape[0], 256))
        for s in range(tab.shape[0]):
            t = tab[s]
            A = t[16:32].reshape(4, 4); B = t[32:48].reshape(4, 4); C = t[48:64].reshape(4, 4)
            D = t[64:80].reshape(4, 4); AB = t[80:96].reshape(4, 4)
            if t[0] == 0:
                F = t[96:160].reshape(4, 4, 4); S = t[160:224].reshape(4, 4, 4)
                e = np.einsum("ax,yb,xyp,pq,qzr,zc,rd->abcd", A, B, F, AB, S, C, D) / 4
            else:
                DD = t[224:480].reshape(4, 4, 4, 4)
                e = np.einsum("ax,yb,zc,xyzr,rd->abcd", A, B, C, DD, D) / 4
            if t[1] == 1:
                e = e.transpose(0, 2, 1, 3)
            elif t[1] == 2:
                e = e.transpose(2, 0, 1, 3)
            out[s] = e.reshape(-1)
        return out
