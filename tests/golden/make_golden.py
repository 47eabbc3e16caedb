#!/usr/bin/env python3
"""Generate the golden fixtures under tests/golden/ from the READ-ONLY reference.

Runs only in the build container (the reference does not exist on the GPU box).  The
reference is pure Python + numba; numba/Biopython are not installed here, so it is imported
under the stand-in package in tests/golden/_shim (identity decorators, dict/list containers).
Under the shim the reference runs as plain CPython + NumPy: `viterbi` and the model build
are not numba-compiled in the reference either (optimizer.py:305, vanloan.py:392), so those
outputs are the reference's own semantics; `forward`/`backward` lose numba's compilation but
keep their arithmetic (optimizer.py:165-213).

Fixtures are DATA only (inputs + expected outputs), written as .npz:

  alphabet.npz          625 observed symbols and the `order` expansion table
                        (read_data.py:6-24, 46-67)
  model_<tag>.npz       a, b, pi, hidden state tuples from trans_emiss_calc
                        (get_trans_emiss.py:8-170) for a parameter set
  sweep_<tag>.npz       an HMM (a, b, pi), seeded blocks of observed symbols and the
                        reference's forward_loglik / viterbi+backtrack_viterbi / post_prob
                        outputs (optimizer.py:145-354)
  expm_kat.npz          reference expm (expm.py:9-167) on matrices hitting every Pade branch
  derive_times.json     the arguments optimization_wrapper (optimizer.py:396-557) passes to
                        trans_emiss_calc for every time-parameter case, captured by
                        replacing trans_emiss_calc in the imported reference module
  model_int_<tag>.npz   a, b, pi, hidden state tuples from the introgression model build
                        trans_emiss_calc_introgression (int_get_trans_emiss.py:9-185); ray
                        (int_get_tab.py:5) is replaced by the standard library's process
                        pool in tests/golden/_shim/ray
  int_derive_times.json the arguments optimization_wrapper_introgression
                        (int_optimizer.py:397-548) passes to trans_emiss_calc_introgression
                        for every time-parameter case (captured like derive_times.json)
  int_statespace.json   the CTMC state spaces and rate-symbol matrices load_trans_mat(1..3)
                        returns (int_load_trans_mat.py:6-41), as sets of transitions
  coal_tables.npz       the reference's one- and two-coalescence tables
                        p_b_c_given_a_JC69_analytical / p_b_c_d_given_a_JC69_analytical
                        (get_emission_prob_mat.py:95-118, 400-424: closed forms summed in
                        the reference's order) at a few (t, mu, k)

Usage:  python tests/golden/make_golden.py alphabet|sweeps|expm|model|intmodel <tag> ...|intspace|coal
"""
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF_SRC = "/root/reference/src"


def _import_reference():
    sys.path.insert(0, os.path.join(HERE, "_shim"))
    sys.path.insert(0, REF_SRC)
    import itrails.ncpu as ncpu

    ncpu.update_n_cpu(int(os.environ.get("GOLDEN_NCPU", "1")))
    return ncpu


# --------------------------------------------------------------------------------------
# parameter sets (user units, like example_config.yaml); scaled exactly as
# optimizer.py:396-557 does for the {t_1} case before calling trans_emiss_calc
# --------------------------------------------------------------------------------------
PARAMS = {
    # the KAT set recorded in SURVEY.md 8(c)
    "kat": dict(mu=2e-8, N_AB=50000.0, N_ABC=50000.0, t_1=240000.0, t_2=40000.0,
                t_upper=745069.3855, r=1e-8),
    # a second, asymmetric set: different Ne, faster recombination
    "alt": dict(mu=1.5e-8, N_AB=30000.0, N_ABC=70000.0, t_1=180000.0, t_2=60000.0,
                t_upper=500000.0, r=2.5e-8),
}

MODELS = {
    # tag: (param set, n_int_AB, n_int_ABC)
    "kat_1_1": ("kat", 1, 1),
    "kat_2_2": ("kat", 2, 2),
    "kat_3_3": ("kat", 3, 3),
    "alt_2_3": ("alt", 2, 3),
    "alt_3_2": ("alt", 3, 2),
    "kat_4_4": ("kat", 4, 4),
    "kat_5_5": ("kat", 5, 5),
    "kat_7_7": ("kat", 7, 7),
}


def scaled_args(pset, n_ab, n_abc):
    from itrails.cutpoints import cutpoints_ABC

    p = PARAMS[pset]
    mu = p["mu"]
    t_1 = p["t_1"] * mu
    t_2 = p["t_2"] * mu
    t_upper = p["t_upper"] * mu
    N_AB = p["N_AB"] * mu
    N_ABC = p["N_ABC"] * mu
    r = p["r"] / mu
    cut_ABC = cutpoints_ABC(n_abc, 1)
    t_A = t_B = t_1
    t_C = t_1 + t_2
    t_out = t_1 + t_2 + cut_ABC[n_abc - 1] * N_ABC + t_upper + 2 * N_ABC
    return dict(t_A=t_A, t_B=t_B, t_C=t_C, t_2=t_2, t_upper=t_upper, t_out=t_out,
                N_AB=N_AB, N_ABC=N_ABC, r=r, n_int_AB=n_ab, n_int_ABC=n_abc)


def cmd_alphabet():
    _import_reference()
    from itrails.read_data import get_idx_state, get_obs_state_dct

    names = get_obs_state_dct()
    order = [np.asarray(get_idx_state(i), dtype=np.int64) for i in range(625)]
    off = np.zeros(626, dtype=np.int64)
    off[1:] = np.cumsum([len(o) for o in order])
    np.savez_compressed(
        os.path.join(HERE, "alphabet.npz"),
        names=np.array(names),
        order_flat=np.concatenate(order),
        order_off=off,
    )
    print("alphabet.npz written")


def cmd_model(tag):
    _import_reference()
    from itrails.get_trans_emiss import trans_emiss_calc

    pset, n_ab, n_abc = MODELS[tag]
    kw = scaled_args(pset, n_ab, n_abc)
    t0 = time.time()
    a, b, pi, hidden, observed = trans_emiss_calc(
        kw["t_A"], kw["t_B"], kw["t_C"], kw["t_2"], kw["t_upper"], kw["t_out"],
        kw["N_AB"], kw["N_ABC"], kw["r"], kw["n_int_AB"], kw["n_int_ABC"],
        "standard", "standard")
    dt = time.time() - t0
    hidden_arr = np.array([hidden[i] for i in range(len(hidden))], dtype=np.int64)
    obs_names = np.array([observed[i] for i in range(len(observed))])
    np.savez_compressed(
        os.path.join(HERE, f"model_{tag}.npz"),
        a=a, b=b, pi=pi, hidden=hidden_arr, observed=obs_names,
        args=np.array([kw[k] for k in ("t_A", "t_B", "t_C", "t_2", "t_upper", "t_out",
                                       "N_AB", "N_ABC", "r")]),
        n_int=np.array([n_ab, n_abc]), build_seconds=np.array(dt),
    )
    print(f"model_{tag}.npz written: N={a.shape[0]} in {dt:.1f}s")


# --------------------------------------------------------------------------------------
# introgression model (int_get_trans_emiss.py)
# --------------------------------------------------------------------------------------
INT_PARAMS = {
    # the KAT set plus an introgression 20 kyr before the first speciation: {t_1} case of
    # int_optimizer.py:504-520 (t_B = t_C = t_1 - t_m)
    "ikat": dict(mu=2e-8, N_AB=50000.0, N_BC=40000.0, N_ABC=50000.0, t_1=240000.0,
                 t_m=20000.0, t_2=40000.0, t_upper=745069.3855, r=1e-8, m=0.1),
    # asymmetric: {t_A, t_B, t_C} case (int_optimizer.py:406-419), other Ne, more migration
    "ialt": dict(mu=1.5e-8, N_AB=30000.0, N_BC=60000.0, N_ABC=70000.0, t_A=180000.0,
                 t_B=150000.0, t_C=165000.0, t_m=25000.0, t_2=60000.0, t_upper=500000.0,
                 r=2.5e-8, m=0.3),
}
INT_MODELS = {
    "ikat_1_1": ("ikat", 1, 1), "ikat_2_2": ("ikat", 2, 2), "ikat_3_3": ("ikat", 3, 3),
    "ialt_2_3": ("ialt", 2, 3), "ialt_3_2": ("ialt", 3, 2), "ikat_1_3": ("ikat", 1, 3),
    "ikat_4_4": ("ikat", 4, 4), "ikat_5_5": ("ikat", 5, 5),
}
INT_ARGS = ("t_A", "t_B", "t_C", "t_2", "t_upper", "t_out", "t_m", "N_AB", "N_BC", "N_ABC",
            "r", "m")


def int_scaled_args(pset, n_ab, n_abc):
    """mu-scaled arguments of trans_emiss_calc_introgression, derived like
    optimization_wrapper_introgression (int_optimizer.py:404-529)."""
    from itrails.cutpoints import cutpoints_ABC

    p = INT_PARAMS[pset]
    mu = p["mu"]
    d = {k: v * mu for k, v in p.items() if k not in ("mu", "r", "m")}
    d["r"] = p["r"] / mu
    d["m"] = p["m"]
    cut_ABC = cutpoints_ABC(n_abc, 1)
    if "t_1" in d:
        d["t_A"] = d["t_1"]
        d["t_B"] = d["t_C"] = d["t_1"] - d["t_m"]
        d["t_out"] = (d["t_1"] + d["t_2"] + cut_ABC[n_abc - 1] * d["N_ABC"] + d["t_upper"]
                      + 2 * d["N_ABC"])
        d.pop("t_1")
    else:
        d["t_out"] = (((d["t_A"] + (d["t_B"] + d["t_m"])) / 2 + d["t_2"])
                      + (d["t_C"] + d["t_m"] + d["t_2"]) / 2
                      + cut_ABC[n_abc - 1] * d["N_ABC"] + d["t_upper"] + 2 * d["N_ABC"])
    return d


def cmd_intmodel(tag):
    import tempfile

    _import_reference()
    from itrails.int_get_trans_emiss import trans_emiss_calc_introgression

    pset, n_ab, n_abc = INT_MODELS[tag]
    d = int_scaled_args(pset, n_ab, n_abc)
    t0 = time.time()
    a, b, pi, hidden, observed = trans_emiss_calc_introgression(
        *[d[k] for k in INT_ARGS], n_ab, n_abc, "standard", "standard", tempfile.mkdtemp())
    dt = time.time() - t0
    hidden_arr = np.array([hidden[i] for i in range(len(hidden))], dtype=np.int64)
    obs_names = np.array([observed[i] for i in range(len(observed))])
    np.savez_compressed(
        os.path.join(HERE, f"model_int_{tag}.npz"),
        a=a, b=b, pi=pi, hidden=hidden_arr, observed=obs_names,
        args=np.array([d[k] for k in INT_ARGS]), n_int=np.array([n_ab, n_abc]),
        build_seconds=np.array(dt),
    )
    print(f"model_int_{tag}.npz written: N={a.shape[0]} in {dt:.1f}s")


def cmd_intspace():
    import json
    from ast import literal_eval

    _import_reference()
    from itrails.int_load_trans_mat import load_trans_mat

    out = {}
    for n_seq in (1, 2, 3):
        mat, names = load_trans_mat(n_seq)
        states = [repr(literal_eval(s)) for s in names]
        trans = sorted([states[i], states[j], str(mat[i, j])]
                       for i in range(len(states)) for j in range(len(states))
                       if str(mat[i, j]) != "0")
        out[str(n_seq)] = {"absorbing_last_two": states[-2:], "first": states[:2],
                           "n_states": len(states), "transitions": trans}
    # the hand-written chain of one missing B lineage (int_get_joint_prob_mat.py:306-339)
    from itrails.int_get_joint_prob_mat import load_trans_mat_miss

    mat, names = load_trans_mat_miss()
    out["miss"] = {"states": [repr(literal_eval(s)) for s in names],
                   "symbols": [[str(v) for v in row] for row in mat]}
    with open(os.path.join(HERE, "int_statespace.json"), "w") as f:
        json.dump(out, f)
    print("int_statespace.json written")


# --------------------------------------------------------------------------------------
# sweeps
# --------------------------------------------------------------------------------------
def synthetic_hmm(rng, n, stay=(0.93, 0.995), sharp=0.3):
    """Random HMM with a strong diagonal and distinct per-state emissions, so that the
    Viterbi path switches states often (the reference models barely switch)."""
    a = rng.random((n, n)) ** 3
    np.fill_diagonal(a, 0.0)
    a /= a.sum(1, keepdims=True)
    d = rng.uniform(*stay, size=n)
    a = a * (1 - d)[:, None]
    a[np.arange(n), np.arange(n)] = d
    b = rng.dirichlet(np.full(256, sharp), size=n)
    pi = rng.dirichlet(np.ones(n))
    return a, b, pi


def sample_blocks(rng, a, b, pi, lengths, names, p_n=0.02, p_gap=0.01):
    """Sample hidden paths from a and 4-species columns from b; inject N and '-' (-> N,
    read_data.py:106) at the given rates.  Returns concatenated obs indices + offsets."""
    n = a.shape[0]
    index = {s: i for i, s in enumerate(names)}
    letters = np.array(list("ACTG"))
    obs = []
    for T in lengths:
        s = rng.choice(n, p=pi / pi.sum())
        for t in range(T):
            if t:
                s = rng.choice(n, p=a[s])
            c = rng.choice(256, p=b[s] / b[s].sum())
            col = [letters[(c >> (2 * (3 - k))) & 3] for k in range(4)]
            for k in range(4):
                u = rng.random()
                if u < p_n + p_gap:
                    col[k] = "N"
            obs.append(index["".join(col)])
    off = np.zeros(len(lengths) + 1, dtype=np.int64)
    off[1:] = np.cumsum(lengths)
    return np.array(obs, dtype=np.uint16), off


def run_reference_sweeps(a, b, pi, obs, off, post_rows_every):
    from itrails.optimizer import backtrack_viterbi, forward_loglik, post_prob, viterbi
    from itrails.read_data import get_idx_state

    order = [get_idx_state(i) for i in range(625)]
    ll, paths, post_idx, post_val = [], [], [], []
    for k in range(len(off) - 1):
        V = obs[off[k]:off[k + 1]].astype(np.int64)
        ll.append(forward_loglik(a, b, pi, V, order))
        om, prev = viterbi(a, b, pi, V, order)
        paths.append(backtrack_viterbi(om, prev))
        pp = post_prob(a, b, pi, V, order)
        rows = np.unique(np.r_[0, np.arange(0, len(V), post_rows_every), len(V) - 1])
        post_idx.append(rows + off[k])
        post_val.append(pp[rows])
    return (np.array(ll), np.concatenate(paths), np.concatenate(post_idx),
            np.concatenate(post_val))


def cmd_sweeps(only=()):
    _import_reference()
    from itrails.read_data import get_obs_state_dct

    names = get_obs_state_dct()
    cases = []
    rng = np.random.default_rng(20260115)
    # synthetic HMMs: small, odd, around a wavefront, and the two BASELINE sizes
    for n, lengths in [
        (4, [1, 2, 3, 50, 700]),
        (13, [5, 1, 400, 1300]),
        (27, [1, 64, 900, 2000]),
        (65, [2, 300, 1700]),
        (70, [1, 33, 1500, 2500]),
        (133, [7, 600, 1400]),
    ]:
        a, b, pi = synthetic_hmm(rng, n)
        cases.append((f"syn{n}", a, b, pi, lengths))
    # real models from the reference model build (fixtures produced by `model`)
    for tag, lengths in [("kat_3_3", [1, 5, 3000, 4000]), ("kat_5_5", [2, 2500, 3500])]:
        f = os.path.join(HERE, f"model_{tag}.npz")
        if not os.path.exists(f):
            print("skip", tag, "(model fixture missing)")
            continue
        m = np.load(f)
        cases.append((tag, m["a"], m["b"], m["pi"], lengths))
    for tag, a, b, pi, lengths in cases:
        t0 = time.time()
        # every case draws from its own stream so a subset can be regenerated alone
        rng = np.random.default_rng([20260115, sum(map(ord, tag))])
        obs, off = sample_blocks(rng, a, b, pi, lengths, names)
        if only and tag not in only:
            continue
        ll, path, pidx, pval = run_reference_sweeps(a, b, pi, obs, off, post_rows_every=37)
        np.savez_compressed(
            os.path.join(HERE, f"sweep_{tag}.npz"),
            a=a, b=b, pi=pi, obs=obs, off=off, loglik=ll,
            path=path.astype(np.int16), post_rows=pidx, post=pval)
        switches = int((np.diff(path) != 0).sum())
        print(f"sweep_{tag}.npz: N={a.shape[0]} cols={off[-1]} switches={switches} "
              f"{time.time() - t0:.1f}s")


def cmd_expm():
    _import_reference()
    from itrails.expm import expm

    rng = np.random.default_rng(7)
    out = {}
    # 1-norms around every branch threshold of expm.py:16-140
    # (theta = 1.5e-2, 2.5e-1, 9.5e-1, 2.1, 5.4; beyond -> scaling & squaring)
    targets = (1e-3, 1.4e-2, 0.2, 0.9, 2.0, 5.0, 9.0, 40.0, 300.0)
    for n in (2, 4, 15, 31, 203):
        mats, outs = [], []
        for target in (targets if n < 100 else targets[3::3]):
            q = rng.random((n, n))
            np.fill_diagonal(q, 0.0)
            np.fill_diagonal(q, -q.sum(1))  # a rate matrix, like trans_mat.py:487-508
            q *= target / np.abs(q).sum(0).max()
            mats.append(q.copy())
            outs.append(expm(q.copy()))
        out[f"A_{n}"] = np.array(mats)
        out[f"E_{n}"] = np.array(outs)
    out["targets"] = np.array(targets)
    np.savez_compressed(os.path.join(HERE, "expm_kat.npz"), **out)
    print("expm_kat.npz written")


class _Captured(Exception):
    pass


def cmd_derive():
    """Every case of optimizer.py:419-541, t_out derived and fixed, two ABC interval
    counts; the reference's optimization_wrapper runs until it calls trans_emiss_calc."""
    import json
    import tempfile

    _import_reference()
    import itrails.optimizer as ref_opt

    def capture(*args):
        raise _Captured(args)

    ref_opt.trans_emiss_calc = capture
    mu = 2e-8
    base = dict(t_1=240000.0, t_A=250000.0, t_B=230000.0, t_C=290000.0, t_2=40000.0,
                t_upper=745069.3855, N_AB=30000.0, N_ABC=50000.0, r=1e-8, t_out=2.5e6)
    cases = [["t_A", "t_B", "t_C"], ["t_1", "t_A"], ["t_1", "t_B"], ["t_1", "t_C"],
             ["t_A", "t_B"], ["t_A", "t_C"], ["t_B", "t_C"], ["t_1"]]
    out = []
    tmp = tempfile.mkdtemp()
    for case in cases:
        for fixed_out in (False, True):
            for n_abc in (3, 5):
                # optimized: the case's times + N_ABC + t_upper; fixed: the rest (mu-scaled)
                names = list(case) + ["N_ABC", "t_upper"]
                d = {"n_int_AB": 3, "n_int_ABC": n_abc, "t_2": base["t_2"] * mu,
                     "N_AB": base["N_AB"] * mu, "r": base["r"] / mu}
                if fixed_out:
                    d["t_out"] = base["t_out"] * mu
                args = [base[k] * mu for k in names]
                try:
                    ref_opt.optimization_wrapper(np.array(args), names, frozenset(case), d,
                                                 [], os.path.join(tmp, "x"),
                                                 {"Nfeval": 0, "time": 0.0})
                    raise RuntimeError("trans_emiss_calc was not reached")
                except _Captured as c:
                    got = list(c.args[0])
                out.append({"case": case, "names": names, "args": args, "fixed": d,
                            "trans_emiss_args": [g if not isinstance(g, np.ndarray) else g.tolist()
                                                 for g in got]})
    with open(os.path.join(HERE, "derive_times.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(f"derive_times.json written ({len(out)} cases)")


def cmd_intderive():
    """Every case of int_optimizer.py:404-529, t_out derived and fixed, two ABC interval
    counts; the reference's wrapper runs until it calls trans_emiss_calc_introgression."""
    import json
    import tempfile

    _import_reference()
    import itrails.int_optimizer as ref_opt

    def capture(*args):
        raise _Captured(args)

    ref_opt.trans_emiss_calc_introgression = capture
    mu = 2e-8
    base = dict(t_1=240000.0, t_A=250000.0, t_B=210000.0, t_C=230000.0, t_2=40000.0,
                t_m=15000.0, t_upper=745069.3855, N_AB=30000.0, N_BC=45000.0, N_ABC=50000.0,
                r=1e-8, m=0.2, t_out=2.5e6)
    cases = [["t_A", "t_B", "t_C"], ["t_1", "t_A"], ["t_1", "t_B"], ["t_1", "t_C"],
             ["t_A", "t_B"], ["t_A", "t_C"], ["t_B", "t_C"], ["t_1"]]
    out = []
    tmp = tempfile.mkdtemp()
    for case in cases:
        for fixed_out in (False, True):
            for n_abc in (3, 5):
                names = list(case) + ["N_ABC", "t_upper", "t_m", "m"]
                d = {"n_int_AB": 3, "n_int_ABC": n_abc, "t_2": base["t_2"] * mu,
                     "N_AB": base["N_AB"] * mu, "N_BC": base["N_BC"] * mu,
                     "r": base["r"] / mu}
                if fixed_out:
                    d["t_out"] = base["t_out"] * mu
                args = [base[k] * mu for k in names]
                try:
                    ref_opt.optimization_wrapper_introgression(
                        np.array(args), names, frozenset(case), d, [],
                        os.path.join(tmp, "x"),
                        {"Nfeval": 1, "time": 0.0, "tmp_path": tmp})
                    raise RuntimeError("trans_emiss_calc_introgression was not reached")
                except _Captured as c:
                    got = list(c.args[0])
                out.append({"case": case, "names": names, "args": args, "fixed": d,
                            "trans_emiss_args": [g if not isinstance(g, np.ndarray) else g.tolist()
                                                 for g in got]})
    with open(os.path.join(HERE, "int_derive_times.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(f"int_derive_times.json written ({len(out)} cases)")


COAL_CASES = [(0.8, 0.3, 1.3), (0.4054651081081643, 4 / 3000, 1.0), (14.90138771, 4 / 3000, 1.0), (0.20279819382384456, 4 / 3000, 1.0)]


def cmd_coal():
    _import_reference()
    from itrails.get_emission_prob_mat import (p_b_c_d_given_a_JC69_analytical,
                                               p_b_c_given_a_JC69_analytical)
    nt = "AGCT"
    singles, doubles = [], []
    for t, mu, k in COAL_CASES:
        S = np.zeros((4, 4, 4))
        for a, b, c, v in p_b_c_given_a_JC69_analytical(t, mu, k):
            S[nt.index(a), nt.index(b), nt.index(c)] = v
        D = np.zeros((4, 4, 4, 4))
        for a, b, c, d, v in p_b_c_d_given_a_JC69_analytical(t, mu):
            D[nt.index(a), nt.index(b), nt.index(c), nt.index(d)] = v
        singles.append(S)
        doubles.append(D)
    np.savez(os.path.join(HERE, "coal_tables.npz"), cases=np.array(COAL_CASES),
             single=np.array(singles), double=np.array(doubles))
    print("coal_tables.npz written")


if __name__ == "__main__":
    cmd = sys.argv[1]
    if cmd == "alphabet":
        cmd_alphabet()
    elif cmd == "model":
        for t in sys.argv[2:]:
            cmd_model(t)
    elif cmd == "sweeps":
        cmd_sweeps(tuple(sys.argv[2:]))
    elif cmd == "expm":
        cmd_expm()
    elif cmd == "derive":
        cmd_derive()
    elif cmd == "intmodel":
        for t in sys.argv[2:]:
            cmd_intmodel(t)
    elif cmd == "intspace":
        cmd_intspace()
    elif cmd == "intderive":
        cmd_intderive()
    elif cmd == "coal":
        cmd_coal()
    else:
        raise SystemExit(__doc__)
