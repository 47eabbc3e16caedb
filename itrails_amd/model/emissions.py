"""Emission probabilities of the iTRAILS hidden states.

Restates get_emission_prob_mat.py:701-1038 and cutpoints.py:5-45.

Per hidden state (topology, i, j) the 256 N-free columns a0 b0 c0 d0 get the probability of
the gene tree: JC69 substitution along every branch and coalescences inside interval i
(and j).  The pieces:

  * branch transition matrices P = expm(sum_k t_k Q_k) with Q = JC69(mu_k)
    (get_emission_prob_mat.py:9-44) — 4x4 exponentials of JC69-form generators, in closed
    form on the host (jc69_propagators);
  * the single-coalescence table F[a][b][c] = sum_d E[ P(a->d, s) P(d->b, s) P(d->c, t-s) ],
    s ~ k e^{-ks} conditioned on s < t (get_emission_prob_mat.py:47-90);
  * the double-coalescence table DD[a][b][c][d] = sum_{e,f} of the analogous two-event
    integral for three lineages (rates 3 then 1, get_emission_prob_mat.py:93-424).
    Both are evaluated here by expanding every JC69 factor 1/4 + (delta - 1/4) e^{-mu tau}
    into exponentials and integrating each term exactly (`_expo_integral`), which gives
    the reference's closed forms to rounding;
  * the 4^6 / 4^4 contraction over ancestral nucleotides and the species re-keying of
    topologies 2 and 3 — the HIP kernel of emission.hip (itr_emission_rows).
"""
from __future__ import annotations

from typing import List, Tuple

import numpy as np
import scipy.special as sc

# ---------------------------------------------------------------------------------------
# cutpoints (cutpoints.py:5-45): quantiles of the (truncated) exponential coalescence time
# ---------------------------------------------------------------------------------------


def cutpoints_AB(n_int_AB: int, t_AB: float, coal_AB: float) -> np.ndarray:
    """truncexpon.ppf(q, b=t_AB*coal_AB, scale=1/coal_AB), q = 0, 1/n, ..., 1."""
    q = np.arange(n_int_AB + 1) / n_int_AB
    scale = 1 / coal_AB
    b = (t_AB - 0) / scale
    out = np.empty(n_int_AB + 1)
    inner = (q > 0) & (q < 1)
    out[inner] = -sc.log1p(q[inner] * sc.expm1(-b)) * scale + 0
    out[q == 0] = 0 * scale + 0
    out[q == 1] = b * scale + 0
    return out


def cutpoints_ABC(n_int_ABC: int, coal_ABC: float) -> np.ndarray:
    """expon.ppf(q, scale=1/coal_ABC), q = 0, 1/n, ..., 1 (last = +inf)."""
    q = np.arange(n_int_ABC + 1) / n_int_ABC
    scale = 1 / coal_ABC
    out = np.empty(n_int_ABC + 1)
    inner = (q > 0) & (q < 1)
    out[inner] = -sc.log1p(-q[inner]) * scale + 0
    out[q == 0] = 0.0
    out[q == 1] = np.inf
    return out


# ---------------------------------------------------------------------------------------
# coalescence integrals
# ---------------------------------------------------------------------------------------
_DELTA = np.eye(4) - 0.25  # JC69: P(x -> y, tau) = 1/4 + (delta_xy - 1/4) e^{-mu tau}


def _phi(lam, t):
    """int_0^t e^{lam s} ds."""
    lam = np.asarray(lam, dtype=np.float64)
    safe = np.where(lam == 0, 1.0, lam)
    return np.where(lam == 0, t, sc.expm1(lam * t) / safe)


def _expo_integral(terms, t):
    """Sum of c * int_0^t e^{lam s} ds over terms [(c, lam)]."""
    return sum(c * _phi(lam, t) for c, lam in terms)


def _single_coeffs():
    """The six coefficient arrays of single_table's integrand (a, b, c, d), without the
    e^{-mu t} factor of the terms that carry it (flag 1)."""
    if "single" not in _COEFFS:
        al = _DELTA[:, None, None, :]   # (a, ., ., d)
        be = _DELTA.T[None, :, None, :]  # (., b, ., d): delta(d, b)
        ga = _DELTA.T[None, None, :, :]  # (., ., c, d): delta(d, c)
        full = lambda x: np.broadcast_to(x, (4, 4, 4, 4)).reshape(-1)  # noqa: E731
        terms = [(1 / 64, 0, 0), (ga / 16, 1, 1), ((al + be) / 16, 0, -1),
                 ((al + be) * ga / 4, 1, 0), (al * be / 4, 0, -2), (al * be * ga, 1, -1)]
        _COEFFS["single"] = (np.stack([full(c) for c, _, _ in terms]),
                             np.array([f for _, f, _ in terms]),
                             np.array([m for _, _, m in terms], dtype=np.float64))
    return _COEFFS["single"]


_COEFFS: dict = {}


def single_table(t: float, mu: float, k: float) -> np.ndarray:
    """F[a, b, c] = sum_d k/(1-e^{-kt}) int_0^t e^{-ks} P(a,d;s) P(d,b;s) P(d,c;t-s) ds
    (p_b_c_given_a_JC69_analytical, get_emission_prob_mat.py:73-90).
    (1/4 + al x)(1/4 + be x)(1/4 + ga e^{-mu t} / x), x = e^{-mu s}, weight e^{-ks}: six
    exponential terms whose coefficient arrays are fixed, so one weighted sum of them."""
    return single_tables([(t, mu, k)])[0]


def single_tables(keys) -> np.ndarray:
    """single_table of every (t, mu, k) in `keys` at once: (K, 4, 4, 4)."""
    C, flag, mpow = _single_coeffs()
    kt = np.asarray(keys, dtype=np.float64).reshape(-1, 3)
    t, mu, k = kt[:, 0:1], kt[:, 1:2], kt[:, 2:3]
    emt = np.exp(-mu * t)
    w = np.where(flag == 1, emt, 1.0) * _phi(-k + mu * mpow, t)
    val = k * (w @ C) / (1 - np.exp(-(k * t)))
    return val.reshape(-1, 4, 4, 4, 4).sum(axis=4)


def _double_coeffs():
    """The 24 coefficient arrays of double_table's integrand (a, b, c, d, e, f) with their
    exponents, without the e^{-mu t} factor (flag v = -1)."""
    if "double" not in _COEFFS:
        D = _DELTA
        al = D[:, None, None, None, :, None]          # delta(a, e)
        be = D.T[None, :, None, None, :, None]        # delta(e, b)
        ga = D[None, None, None, None, :, :]          # delta(e, f)
        de = D.T[None, None, :, None, None, :]        # delta(f, c)
        ep = D.T[None, None, None, :, None, :]        # delta(f, d)
        A = [(1 / 16, 0), ((al + be) / 4, 1), (al * be, 2)]   # coefficient, power of y1
        G = [(1 / 4, 0), (ga, 1)]                             # y2^q y1^-q
        Dl = [(1 / 4, 0), (de, 1)]                            # y2^u
        Ep = [(1 / 4, 0), (ep, -1)]                           # y2^-v (x e^{-mu t})
        cs, pq, quv, flag = [], [], [], []
        for ca, p in A:
            for cg, q in G:
                for cd, u in Dl:
                    for ce, v in Ep:
                        cs.append(np.broadcast_to(ca * cg * cd * ce, (4,) * 6).reshape(-1))
                        pq.append(p - q)
                        quv.append(q + u + v)
                        flag.append(v == -1)
        _COEFFS["double"] = (np.stack(cs), np.array(pq, dtype=np.float64),
                             np.array(quv, dtype=np.float64), np.array(flag))
    return _COEFFS["double"]


def double_table(t: float, mu: float) -> np.ndarray:
    """DD[a, b, c, d] = sum_{e, f} of the two-coalescence integral: (a, b) -> e at s1
    (rate 3), (e, c) -> f at s2 > s1 (rate 1), f -> d over t - s2; normalised by the
    probability that both happen before t (JC69_analytical_integral_double,
    get_emission_prob_mat.py:93-424, summed as in 427-441).
    Factors in s1, s2: e^{-2 s1} e^{-s2}, (1/4 + al y1)(1/4 + be y1), (1/4 + ga y2 / y1),
    (1/4 + de y2), (1/4 + ep e^{-mu t} / y2) with y1 = e^{-mu s1}, y2 = e^{-mu s2}: 24
    exponential terms with fixed coefficient arrays, one weighted sum of them."""
    return double_tables([(t, mu)])[0]


def double_tables(keys) -> np.ndarray:
    """double_table of every (t, mu) in `keys` at once: (K, 4, 4, 4, 4)."""
    C, pq, quv, flag = _double_coeffs()
    tm = np.asarray(keys, dtype=np.float64).reshape(-1, 2)
    t, mu = tm[:, 0:1], tm[:, 1:2]
    emt = np.exp(-mu * t)
    lam1 = -2.0 - mu * pq
    lam2 = -1.0 - mu * quv
    # int_0^t e^{lam2 s2} int_0^{s2} e^{lam1 s1} ds1 ds2 (lam1 = 0 / lam2 = 0: the limits)
    with np.errstate(divide="ignore", invalid="ignore"):
        l1 = np.where(lam1 == 0.0, 1.0, lam1)
        l2 = np.where(lam2 == 0.0, 1.0, lam2)
        inner = np.where(lam1 != 0.0, (_phi(lam1 + lam2, t) - _phi(lam2, t)) / l1,
                         np.where(lam2 != 0.0,
                                  t * np.exp(lam2 * t) / l2 - sc.expm1(lam2 * t) / l2 ** 2,
                                  t * t / 2))
    w = np.where(flag, emt, 1.0) * inner
    den = 1 + 0.5 / np.exp(3 * t) - 1.5 / np.exp(t)
    val = (3 * (w @ C) / den).reshape(-1, 4, 4, 4, 4, 16)
    # the 16 (e, f) terms summed one after another, e outer, like the reference's cumsum
    # (get_emission_prob_mat.py:417-423); NumPy's sum over 16 would pair them
    out = val[..., 0].copy()
    for i in range(1, 16):
        out = out + val[..., i]
    return out


def jc69_rate(mu: float) -> np.ndarray:
    return np.full((4, 4), mu / 4) - np.diag([mu, mu, mu, mu])


def branch_generator(ts, mus) -> tuple:
    """sum_k t_k Q_k (p_b_given_a, get_emission_prob_mat.py:22-44), exponentiated later, as
    its two distinct entries (off-diagonal, diagonal): every Q_k = jc69_rate(mu_k) has one
    off-diagonal value mu/4 and one diagonal value mu/4 - mu, so the elementwise sum is two
    scalar sums in the same order (bit-equal); jc69_propagators exponentiates them,
    generator_matrices expands them."""
    off = 0.0
    dg = 0.0
    for t, mu in zip(ts, mus):
        q = mu / 4
        off = off + t * q
        dg = dg + t * (q - mu)
    return (off, dg)


def jc69_propagators(gens) -> np.ndarray:
    """(G, 4, 4) expm of the branch_generator pairs in closed form: a generator with every
    off-diagonal entry a and every diagonal entry d is a J + (d - a) I (J all ones), so its
    exponential is e^{d-a} (I + (e^{4a} - 1) / 4 J).  Agrees with expm.py's Pade evaluation
    of the same matrices to ~2e-15 relative (the emission bar is 1e-8), and takes no device
    round trip in the middle of the build."""
    g = np.asarray(gens, dtype=np.float64).reshape(-1, 2)
    a = g[:, 0, None, None]
    return np.exp(g[:, 1, None, None] - a) * (np.eye(4) + np.expm1(4.0 * a) / 4.0)


def generator_matrices(gens) -> np.ndarray:
    """(G, 4, 4) matrices of branch_generator pairs: off-diagonal entries `off`, diagonal `dg`."""
    g = np.asarray(gens, dtype=np.float64).reshape(-1, 2)
    out = np.empty((g.shape[0], 4, 4))
    out[:] = g[:, 0, None, None]
    d = np.arange(4)
    out[:, d, d] = g[:, 1, None]
    return out


# ---------------------------------------------------------------------------------------
# per-state specifications (get_emission_prob_mat.py:701-1038)
# ---------------------------------------------------------------------------------------
ET_STRIDE = 512
ET_KIND, ET_PERM, ET_A, ET_B, ET_C, ET_D, ET_AB, ET_F, ET_S, ET_DD = 0, 1, 16, 32, 48, 64, 80, 96, 160, 224


def state_specs(t_A, t_B, t_AB, t_C, t_upper, t_out, coal_AB, coal_ABC, n_int_AB,
                n_int_ABC, mu_A, mu_B, mu_C, mu_D, mu_AB, mu_ABC, cut_AB, cut_ABC):
    """One spec per hidden state, in the reference's generation order:
    (state, kind, perm, gens, first, second, dbl) with gens = branch generators for
    a, b, c, d, ab (b, c and d use the reversed vectors, get_emission_prob_mat.py:612-635)."""
    n = n_int_ABC
    specs = []

    def d_vec(jj):
        add = t_upper + cut_ABC[n - 1] - cut_ABC[jj + 1] if jj != n - 1 else 0
        return [t_out, add], [mu_D, mu_ABC]

    def rev(v):
        return list(reversed(v[0])), list(reversed(v[1]))

    def single(a, b, c, ab, first, second, d, state, perm):
        gens = [branch_generator(*a), branch_generator(*rev(b)), branch_generator(*rev(c)),
                branch_generator(*rev(d)), branch_generator(*ab)]
        specs.append((state, 0, perm, gens, first, second, None))

    def double(a, b, c, tt, d, state, perm):
        gens = [branch_generator(*a), branch_generator(*rev(b)), branch_generator(*rev(c)),
                branch_generator(*rev(d)), None]
        specs.append((state, 1, perm, gens, None, None, (tt, mu_ABC)))

    for i in range(n):
        for j in range(i + 1, n):
            a = ([t_A, t_AB, cut_ABC[i]], [mu_A, mu_AB, mu_ABC])
            b = ([t_B, t_AB, cut_ABC[i]], [mu_B, mu_AB, mu_ABC])
            c = ([t_C, cut_ABC[i]], [mu_C, mu_ABC])
            ab = ([cut_ABC[j] - cut_ABC[i + 1]], [mu_ABC])
            first = (cut_ABC[i + 1] - cut_ABC[i], mu_ABC, coal_ABC)
            second = ((cut_ABC[j + 1] - cut_ABC[j]) if j != n - 1 else t_upper, mu_ABC,
                      coal_ABC)
            d = d_vec(j)
            single(a, b, c, ab, first, second, d, (1, i, j), 0)
            single(a, c, b, ab, first, second, d, (2, i, j), 1)
            single(b, c, a, ab, first, second, d, (3, i, j), 2)
    for i in range(n):
        a = ([t_A, t_AB, cut_ABC[i]], [mu_A, mu_AB, mu_ABC])
        b = ([t_B, t_AB, cut_ABC[i]], [mu_B, mu_AB, mu_ABC])
        c = ([t_C, cut_ABC[i]], [mu_C, mu_ABC])
        tt = (cut_ABC[i + 1] - cut_ABC[i]) if i != n - 1 else t_upper
        d = d_vec(i)
        double(a, b, c, tt, d, (1, i, i), 0)
        double(a, c, b, tt, d, (2, i, i), 1)
        double(b, c, a, tt, d, (3, i, i), 2)
    for i in range(n_int_AB):
        for j in range(n):
            a = ([t_A, cut_AB[i]], [mu_A, mu_AB])
            b = ([t_B, cut_AB[i]], [mu_B, mu_AB])
            c = ([t_C, cut_ABC[j]], [mu_C, mu_ABC])
            ab = ([t_AB - cut_AB[i + 1], cut_ABC[j]], [mu_AB, mu_ABC])
            first = (cut_AB[i + 1] - cut_AB[i], mu_AB, coal_AB)
            second = ((cut_ABC[j + 1] - cut_ABC[j]) if j != n - 1 else t_upper, mu_ABC,
                      coal_ABC)
            single(a, b, c, ab, first, second, d_vec(j), (0, i, j), 0)
    return specs


def emission_rows(specs, la=None) -> Tuple[List[tuple], np.ndarray]:
    """(states, b) with b[s] the 256 emission probabilities of specs[s]: the branch
    exponentials in closed form and the coalescence tables on the host, the contraction on
    the GPU (itr_emission_rows)."""
    if la is None:
        from .linalg import DeviceLinalg
        la = DeviceLinalg()
    gens, where = [], []
    for s, spec in enumerate(specs):
        for g, m in enumerate(spec[3]):
            if m is not None:
                where.append((s, g))
                gens.append(m)
    P = jc69_propagators(gens)
    tab = np.zeros((len(specs), ET_STRIDE))
    slot = np.array([ET_A, ET_B, ET_C, ET_D, ET_AB])
    if where:
        wi = np.asarray(where, dtype=np.int64)
        cols = slot[wi[:, 1]][:, None] + np.arange(16)
        tab[wi[:, 0:1], cols] = P.reshape(len(P), 16)
    # the distinct coalescence tables of the build, each kind in one vectorised evaluation
    skeys = list(dict.fromkeys(k for sp in specs if sp[1] == 0 for k in (sp[4], sp[5])))
    dkeys = list(dict.fromkeys(sp[6] for sp in specs if sp[1] != 0))
    cache = {}
    if skeys:
        cache.update(zip(skeys, single_tables(skeys).reshape(len(skeys), 64)))
    if dkeys:
        cache.update(zip(dkeys, double_tables(dkeys).reshape(len(dkeys), 256)))
    for s, (state, kind, perm, _, first, second, dbl) in enumerate(specs):
        tab[s, ET_KIND] = kind
        tab[s, ET_PERM] = perm
        if kind == 0:
            tab[s, ET_F:ET_F + 64] = cache[first]
            tab[s, ET_S:ET_S + 64] = cache[second]
        else:
            tab[s, ET_DD:ET_DD + 256] = cache[dbl]
    return [sp[0] for sp in specs], la.emission_rows(tab)
