"""The introgression entry points (itrails-int-optimize / -viterbi / -posterior,
workflow_int_*.py): per-case time derivation bit-checked against the arguments the
reference's own optimization_wrapper_introgression passes to
trans_emiss_calc_introgression (tests/golden/int_derive_times.json), the decode/optimize
parameter resolution, and (GPU) the commands end to end."""
import json
import os

import numpy as np
import pytest
import yaml

from itrails_amd import config as C
from itrails_amd.model.emissions import cutpoints_ABC

HERE = os.path.dirname(os.path.abspath(__file__))
SP = ["hg38", "panTro5", "gorGor5", "ponAbe2"]


def _golden():
    with open(os.path.join(HERE, "golden", "int_derive_times.json")) as f:
        return json.load(f)


@pytest.mark.parametrize("k", range(32))
def test_derive_times_int_matches_reference_optimizer(k):
    g = _golden()[k]
    d = dict(g["fixed"])
    for name, v in zip(g["names"], g["args"]):
        d[name] = v
    n = d["n_int_ABC"]
    dd = C.derive_times_int(d, frozenset(g["case"]), cutpoints_ABC(n, 1)[n - 1])
    got = [dd["t_A"], dd["t_B"], dd["t_C"], dd["t_2"], dd["t_upper"], dd["t_out"], dd["t_m"],
           dd["N_AB"], dd["N_BC"], dd["N_ABC"], dd["r"], dd["m"], dd["n_int_AB"],
           dd["n_int_ABC"], "standard", "standard"]
    assert got == g["trans_emiss_args"][:16]  # bit-equal floats
    assert "t_1" not in dd


def _decode_config(tmp_path, **over):
    cfg = {"fixed_parameters": {"mu": 2e-8, "t_1": 240000.0, "t_2": 40000.0, "N_AB": 50000.0,
                                "N_BC": 40000.0, "N_ABC": 50000.0, "r": 1e-8,
                                "t_m": 20000.0, "m": 0.1},
           "optimized_parameters": {"t_upper": 745069.3855},
           "settings": {"input_maf": str(tmp_path / "in.maf"),
                        "output_prefix": str(tmp_path / "out" / "run"),
                        "species_list": SP, "n_int_AB": 2, "n_int_ABC": 2, "n_cpu": 2}}
    for k, v in over.items():
        sec, key = k.split("__")
        if v is None:
            cfg[sec].pop(key, None)
        else:
            cfg[sec][key] = v
    return cfg


def test_resolve_decode_int(tmp_path):
    mu = 2e-8
    s = C.resolve_decode_int(_decode_config(tmp_path))
    d = s.params
    # workflow_int_viterbi.py:446-451: every parameter but r is multiplied by mu — the
    # admixture proportion m included
    assert d["m"] == 0.1 * mu
    assert d["t_m"] == 20000.0 * mu
    assert d["t_A"] == 240000.0 * mu
    assert d["t_B"] == d["t_C"] == 240000.0 * mu - 20000.0 * mu
    cut = cutpoints_ABC(2, 1)
    assert d["t_out"] == (240000.0 * mu + 40000.0 * mu + cut[-2] * 50000.0 * mu
                          + 745069.3855 * mu + 2 * 50000.0 * mu)
    assert s.norm_cut_ABC[-1] == float("inf") and len(s.abs_cut_AB) == 3


def test_resolve_decode_int_proportional(tmp_path):
    cfg = _decode_config(tmp_path, fixed_parameters__t_m=0.25, settings__proportional=True)
    s = C.resolve_decode_int(cfg)
    assert s.params["t_m"] == 240000.0 * 0.25 * 2e-8
    cfg = _decode_config(tmp_path, fixed_parameters__t_m=2.0, settings__proportional=True)
    with pytest.raises(ValueError, match="proportion"):
        C.resolve_decode_int(cfg)
    cfg = _decode_config(tmp_path, fixed_parameters__t_1=None, fixed_parameters__t_A=250000.0,
                         fixed_parameters__t_B=230000.0, fixed_parameters__t_C=230000.0,
                         fixed_parameters__t_m=0.1, settings__proportional=True)
    with pytest.raises(ValueError, match="only supported"):
        C.resolve_decode_int(cfg)


@pytest.mark.parametrize("missing", ["N_BC", "t_m", "m"])
def test_resolve_decode_int_requires_introgression_parameters(tmp_path, missing):
    cfg = _decode_config(tmp_path, **{f"fixed_parameters__{missing}": None})
    with pytest.raises(ValueError, match="N_BC, 't_m', 'm'"):
        C.resolve_decode_int(cfg)


def test_decode_overrides_int(tmp_path):
    from itrails_amd.cli import _decode_parser
    args = _decode_parser("viterbi", intro=True).parse_args(
        ["--t_m", "10000", "--N_BC", "35000", "--m", "0.3"])
    cfg = _decode_config(tmp_path)
    cfg["optimized_parameters"]["m"] = 0.2
    cfg = C.apply_decode_overrides(cfg, args)
    assert cfg["fixed_parameters"]["t_m"] == 10000.0
    assert cfg["fixed_parameters"]["N_BC"] == 35000.0
    assert cfg["fixed_parameters"]["m"] == 0.3 and "m" not in cfg["optimized_parameters"]


def _optimize_config(tmp_path):
    return {"fixed_parameters": {"mu": 2e-8, "t_2": 40000.0, "N_AB": 50000.0, "N_BC": 40000.0,
                                 "r": 1e-8, "t_3": 800000.0},
            "optimized_parameters": {"t_1": [240000, 24000, 2400000],
                                     "N_ABC": [50000, 5000, 500000],
                                     "t_m": [20000, 2000, 200000], "m": [0.1, 0.01, 0.5]},
            "settings": {"input_maf": str(tmp_path / "in.maf"),
                         "output_prefix": str(tmp_path / "o" / "run"), "species_list": SP,
                         "n_int_AB": 1, "n_int_ABC": 1, "n_cpu": 2, "method": "Nelder-Mead"}}


def test_resolve_optimize_int(tmp_path):
    mu = 2e-8
    s = C.resolve_optimize(_optimize_config(tmp_path), intro=True)
    assert s.optim_variables == ["t_1", "N_ABC", "t_m", "m", "t_upper"]
    assert s.optim_list[3] == 0.1 * mu and s.bounds[3] == (0.01 * mu, 0.5 * mu)
    assert s.starting_params["optimized_parameters"]["m"] == [0.1, 0.01, 0.5]
    cfg = _optimize_config(tmp_path)
    cfg["settings"]["proportional"] = True
    with pytest.raises(ValueError, match="not supported in the optimization"):
        C.resolve_optimize(cfg, intro=True)
    cfg = _optimize_config(tmp_path)
    del cfg["optimized_parameters"]["m"]
    with pytest.raises(ValueError, match="'N_BC', 't_m', 'm'"):
        C.resolve_optimize(cfg, intro=True)


def test_hidden_states_int_layout(tmp_path):
    from itrails_amd.writers import write_hidden_states_csv_int
    f = tmp_path / "h.csv"
    write_hidden_states_csv_int(str(f), {0: (0, 0, 0), 1: (4, 1, 0), 2: (1, 0, 1)},
                                [1.0, 2.0, 3.0], [10.0, 20.0, float("inf")])
    assert open(f, newline="").read() == (
        "state_idx,topology,interval_1st_coalescent,interval_2nd_coalescent,shorthand_name\n"
        '0,"({sp1,sp2},sp3)",1.00-2.00,10.00-20.00,"(0, 0, 0)"\n'
        '1,"({sp2,sp3},sp1)",20.00-inf,10.00-20.00,"(4, 1, 0)"\n'
        '2,"((sp1,sp2),sp3)",10.00-20.00,20.00-inf,"(1, 0, 1)"\n')


# ---------------------------------------------------------------------------------------
# GPU: the commands end to end
# ---------------------------------------------------------------------------------------
def _write_maf(path, obs_blocks):
    nt = "ACTG"
    with open(path, "w") as f:
        f.write("##maf version=1\n\n")
        pos = 1000
        for blk in obs_blocks:
            cols = [(nt[s >> 6], nt[(s >> 4) & 3], nt[(s >> 2) & 3], nt[s & 3]) for s in blk]
            f.write("a score=0\n")
            for k, name in enumerate(SP):
                seq = "".join(c[k] for c in cols)
                f.write(f"s {name}.chr1 {pos} {len(seq)} + 100000000 {seq}\n")
            f.write("\n")
            pos += len(blk) + 10


@pytest.fixture
def maf_case(tmp_path):
    rng = np.random.default_rng(5)
    blocks = [rng.integers(0, 256, size=int(n)) for n in (400, 1, 90, 700)]
    blocks[3][100:450] = 5
    path = tmp_path / "aln.maf"
    _write_maf(path, blocks)
    cfg = _decode_config(tmp_path, settings__input_maf=str(path))
    cf = tmp_path / "cfg.yaml"
    with open(cf, "w") as h:
        yaml.dump(cfg, h)
    return tmp_path, cf, blocks


def _model(s):
    from itrails_amd.model.intro import trans_emiss_calc_introgression
    d = s.params
    return trans_emiss_calc_introgression(
        d["t_A"], d["t_B"], d["t_C"], d["t_2"], d["t_upper"], d["t_out"], d["t_m"], d["N_AB"],
        d["N_BC"], d["N_ABC"], d["r"], d["m"], s.n_int_AB, s.n_int_ABC, s.norm_cut_AB,
        s.norm_cut_ABC)


@pytest.mark.gpu
def test_int_viterbi_and_posterior_cli(gpu, maf_case):
    from itrails_amd.cli import int_posterior_main, int_viterbi_main
    from itrails_amd.tables import build_tables
    from itrails_amd.writers import write_viterbi_csv
    from oracle import hmm_oracle as O

    tmp, cf, blocks = maf_case
    int_viterbi_main(["--config-file", str(cf), "--output", str(tmp / "v" / "x")])
    s = C.resolve_decode_int(yaml.safe_load(open(cf)), output_cmd=str(tmp / "chk" / "x"))
    a, b, pi, hidden, _ = _model(s)
    assert any(h[0] == 4 for h in hidden.values())
    obs = np.concatenate(blocks).astype(np.uint16)
    off = np.concatenate([[0], np.cumsum([len(x) for x in blocks])]).astype(np.int64)
    t = build_tables(a, b, pi)
    write_viterbi_csv(str(tmp / "expect.csv"), O.viterbi(t, obs, off).astype(np.uint8),
                      block_off=off)
    assert open(tmp / "v" / "x.viterbi.csv").read() == open(tmp / "expect.csv").read()
    lines = open(tmp / "v" / "x.hidden_states.csv").read().splitlines()
    assert len(lines) == 1 + len(hidden)
    int_posterior_main(["--config-file", str(cf), "--output", str(tmp / "p" / "x")])
    rows = open(tmp / "p" / "x.posterior.csv").read().splitlines()
    got = np.array([[float(v) for v in r.split(",")[2:]] for r in rows[1:]])
    np.testing.assert_allclose(got, O.posterior(t, obs, off), rtol=1e-8, atol=1e-300)


@pytest.mark.gpu
def test_int_optimize_cli_runs(gpu, maf_case, monkeypatch):
    from itrails_amd.cli import int_optimize_main
    import itrails_amd.optimizer as OPT

    tmp, _, _ = maf_case
    cfg = _optimize_config(tmp)
    cfg["settings"]["input_maf"] = str(tmp / "aln.maf")
    cf = tmp / "opt.yaml"
    yaml.dump(cfg, open(cf, "w"))
    orig = OPT.optimizer_introgression
    monkeypatch.setattr(OPT, "optimizer_introgression",
                        lambda **kw: orig(**kw, options={"maxiter": 3, "disp": False}))
    monkeypatch.chdir(tmp)  # the first evaluation writes hidden/observed_states.csv here
    int_optimize_main([str(cf)])
    hist = open(tmp / "o" / "run_optimization_history.csv").read().splitlines()
    assert hist[0] == "n_eval,t_1,N_ABC,t_m,m,t_upper,loglik,time"
    assert len(hist) >= 4
    best = yaml.safe_load(open(tmp / "o" / "run_best_model.yaml"))
    lls = [float(r.split(",")[-2]) for r in hist[1:]]
    assert best["results"]["log_likelihood"] == max(lls)
    assert os.path.exists(tmp / "o" / "run_starting_params.yaml")
    assert open(tmp / "hidden_states.csv").readline() == "idx,hidden\n"
