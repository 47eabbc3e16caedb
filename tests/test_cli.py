"""Command-line surface (itrails_amd.cli / itrails_amd.config) against the reference's
workflow_*.py behaviour.

CPU: parameter resolution — the per-case derivation of t_A/t_B/t_C/t_out is checked
against arguments captured from the reference's own optimization_wrapper
(tests/golden/derive_times.json, make_golden.py derive); the decode / optimize resolution
against values computed by hand from the reference's formulas (workflow_viterbi.py:345-568,
workflow_optimize.py:143-470; the workflow modules themselves cannot be imported here:
their generated _version.py is absent — SURVEY 8c), error messages, and argument parsing.
GPU: itrails-viterbi / itrails-posterior / itrails-optimize end to end on a generated MAF,
checked against the CPU oracle on the same model.
"""
import json
import math
import os

import numpy as np
import pytest
import yaml

from itrails_amd import config as C
from itrails_amd.model.emissions import cutpoints_AB, cutpoints_ABC

HERE = os.path.dirname(os.path.abspath(__file__))
SP = ["hg38", "panTro5", "gorGor5", "ponAbe2"]


def _golden_derive():
    with open(os.path.join(HERE, "golden", "derive_times.json")) as f:
        return json.load(f)


@pytest.mark.parametrize("k", range(32))
def test_derive_times_matches_reference_optimizer(k):
    g = _golden_derive()[k]
    d = dict(g["fixed"])
    for name, v in zip(g["names"], g["args"]):
        d[name] = v
    n = d["n_int_ABC"]
    dd = C.derive_times(d, frozenset(g["case"]), cutpoints_ABC(n, 1)[n - 1])
    got = [dd["t_A"], dd["t_B"], dd["t_C"], dd["t_2"], dd["t_upper"], dd["t_out"], dd["N_AB"],
           dd["N_ABC"], dd["r"], dd["n_int_AB"], dd["n_int_ABC"], "standard", "standard"]
    assert got == g["trans_emiss_args"]  # bit-equal floats
    assert "t_1" not in dd


def _decode_config(tmp_path, **over):
    cfg = {"fixed_parameters": {"mu": 2e-8, "t_1": 240000.0, "t_2": 40000.0, "N_AB": 50000.0,
                                "N_ABC": 50000.0, "r": 1e-8},
           "optimized_parameters": {"t_upper": 745069.3855},
           "settings": {"input_maf": str(tmp_path / "in.maf"),
                        "output_prefix": str(tmp_path / "out" / "run"),
                        "species_list": SP, "n_int_AB": 3, "n_int_ABC": 3, "n_cpu": 2}}
    for k, v in over.items():
        sec, key = k.split("__")
        if v is None:
            cfg[sec].pop(key, None)
        else:
            cfg[sec][key] = v
    return cfg


def test_resolve_decode_kat(tmp_path):
    s = C.resolve_decode(_decode_config(tmp_path), kind="viterbi")
    mu = 2e-8
    p = s.params
    # workflow_viterbi.py:406-424 and the {t_1} row of the case table (552-568)
    assert p["t_A"] == p["t_B"] == 240000.0 * mu
    assert p["t_C"] == 240000.0 * mu + 40000.0 * mu
    assert p["t_upper"] == 745069.3855 * mu and p["r"] == 1e-8 / mu
    cabc = cutpoints_ABC(3, 1)
    assert p["t_out"] == (240000.0 * mu + 40000.0 * mu + cabc[-2] * (50000.0 * mu)
                          + 745069.3855 * mu + 2 * (50000.0 * mu))
    assert s.abs_cut_AB == [240000.0 + x for x in cutpoints_AB(3, 40000.0, 1 / 50000.0)]
    assert s.norm_cut_AB == [(x - 240000.0) / 50000.0 for x in s.abs_cut_AB]
    assert s.norm_cut_ABC == list(cabc) and math.isinf(s.norm_cut_ABC[-1])
    assert s.abs_cut_ABC[:-1] == [x * 50000.0 + 240000.0 + 40000.0 for x in cabc[:-1]]
    assert os.path.isdir(tmp_path / "out") and s.output_prefix == "run"


def test_resolve_decode_t3_and_manual_cutpoints(tmp_path):
    # t_upper fixed is ignored in favour of t_3 (the unreachable branch, quirk 6)
    cfg = _decode_config(tmp_path, optimized_parameters__t_upper=None,
                         fixed_parameters__t_3=800000.0,
                         settings__cutpoints_AB=[240000.0, 250000.0, 260000.0, 280000.0],
                         settings__cutpoints_ABC=[280000.0, 300000.0, 400000.0])
    s = C.resolve_decode(cfg)
    mu = 2e-8
    norm_abc = [(x - 240000.0 - 40000.0) / 50000.0 for x in [280000.0, 300000.0, 400000.0]]
    assert s.norm_cut_ABC[:-1] == norm_abc and math.isinf(s.norm_cut_ABC[-1])
    assert s.params["t_upper"] == (800000.0 - norm_abc[-1] * 50000.0) * mu
    assert s.norm_cut_AB == [(x - 240000.0) / 50000.0 for x in
                             [240000.0, 250000.0, 260000.0, 280000.0]]


@pytest.mark.parametrize("over,msg", [
    ({"fixed_parameters__t_A": 1.0, "fixed_parameters__t_B": 1.0},
     "Invalid combination of time values"),
    ({"fixed_parameters__N_AB": None}, "must be present in optimized or fixed"),
    ({"settings__n_int_AB": 0}, "n_int_AB must be specified"),
    ({"settings__cutpoints_AB": [1.0, 2.0]}, "cutpoints_AB must have n_int_AB + 1 values"),
    ({"optimized_parameters__t_upper": None}, "'t_3' not found"),
    ({"optimized_parameters__t_out": 1.0}, "'t_out' has to be fixed"),
    ({"settings__output_prefix": None}, "Output file not specified"),
    ({"settings__cutpoints_AB": [100.0, 250000.0, 260000.0, 280000.0]},
     "cutpoints_AB must lie within"),
])
def test_resolve_decode_errors(tmp_path, over, msg):
    with pytest.raises(ValueError, match=msg.replace("(", r"\(").replace("+", r"\+")):
        C.resolve_decode(_decode_config(tmp_path, **over))


def test_decode_overrides_move_parameters(tmp_path):
    from itrails_amd.cli import _decode_parser

    cfg = _decode_config(tmp_path)
    args = _decode_parser("viterbi").parse_args(
        ["--t_upper", "700000", "--N_AB", "40000", "--species_list", "a", "b", "c", "d",
         "--n_int_AB", "2"])
    cfg = C.apply_decode_overrides(cfg, args)
    assert "t_upper" not in cfg["optimized_parameters"]
    assert cfg["fixed_parameters"]["t_upper"] == 700000.0
    assert cfg["fixed_parameters"]["N_AB"] == 40000.0
    assert cfg["settings"]["species_list"] == ["a", "b", "c", "d"]
    assert cfg["settings"]["n_int_AB"] == 2
    cfg["fixed_parameters"].pop("mu")
    with pytest.raises(ValueError, match="mu must be specified"):
        C.apply_decode_overrides(cfg, _decode_parser("viterbi").parse_args([]))


def test_decode_cli_without_arguments_exits():
    from itrails_amd.cli import viterbi_main

    with pytest.raises(SystemExit, match="No arguments provided"):
        viterbi_main([])


def _optimize_config(tmp_path):
    cfg = {"fixed_parameters": {"mu": 2e-8},
           "optimized_parameters": {"N_AB": [50000, 5000, 500000],
                                    "N_ABC": [50000, 5000, 500000],
                                    "t_1": [240000, 24000, 2400000],
                                    "t_2": [40000, 4000, 400000],
                                    "t_upper": [745069.3855, 74506.9385, 7450693.8556],
                                    "r": [1e-8, 1e-9, 1e-7]},
           "settings": {"input_maf": str(tmp_path / "in.maf"),
                        "output_prefix": str(tmp_path / "opt" / "run"), "n_cpu": 4,
                        "method": "Nelder-Mead", "species_list": SP, "n_int_AB": 3,
                        "n_int_ABC": 3}}
    return cfg


def test_resolve_optimize_example(tmp_path):
    s = C.resolve_optimize(_optimize_config(tmp_path))
    mu = 2e-8
    # workflow_optimize.py:184-236: time parameters first, then t_2, N_ABC, N_AB, r, t_upper
    assert s.optim_variables == ["t_1", "t_2", "N_ABC", "N_AB", "r", "t_upper"]
    assert s.optim_list == [240000 * mu, 40000 * mu, 50000 * mu, 50000 * mu, 1e-8 / mu,
                            745069.3855 * mu]
    assert s.bounds[4] == (1e-9 / mu, 1e-7 / mu)
    assert s.fixed == {"n_int_AB": 3, "n_int_ABC": 3}
    assert s.case == frozenset(["t_1"]) and s.method == "nelder-mead"
    text = yaml.dump(s.starting_params, default_flow_style=False)
    assert "species_list: [hg38, panTro5, gorGor5, ponAbe2]" in text
    assert "t_1: [" in text and "mu: 2.0e-08" in text
    assert s.best_model["results"] == {"log_likelihood": -math.inf, "iteration": None}


def test_resolve_optimize_t3(tmp_path):
    cfg = _optimize_config(tmp_path)
    del cfg["optimized_parameters"]["t_upper"]
    cfg["optimized_parameters"]["t_3"] = [800000, 700000, 8000000]
    cfg["optimized_parameters"]["N_ABC"] = [50000, 5000, 100000]
    s = C.resolve_optimize(cfg)
    mu = 2e-8
    last = lambda n: cutpoints_ABC(3, 1 / n)[-2]  # noqa: E731
    i = s.optim_variables.index("t_upper")
    assert s.optim_list[i] == (800000 - last(50000)) * mu
    assert s.bounds[i] == ((700000 - last(100000)) * mu, (8000000 - last(5000)) * mu)
    cfg = _optimize_config(tmp_path)
    del cfg["optimized_parameters"]["t_upper"]
    cfg["optimized_parameters"]["t_3"] = [800000, 80000, 8000000]
    with pytest.raises(ValueError, match="cannot be negative"):
        C.resolve_optimize(cfg)


@pytest.mark.parametrize("over,msg", [
    ({"method": "bfgs"}, "Method must be one of"),
    ({"n_int_AB": 0}, "n_int_AB must be a positive integer"),
])
def test_resolve_optimize_errors(tmp_path, over, msg):
    cfg = _optimize_config(tmp_path)
    cfg["settings"].update(over)
    with pytest.raises(ValueError, match=msg):
        C.resolve_optimize(cfg)


def test_start_outside_bounds(tmp_path):
    cfg = _optimize_config(tmp_path)
    cfg["optimized_parameters"]["r"] = [1e-6, 1e-9, 1e-7]
    with pytest.raises(ValueError, match=r"Starting value for 'r'"):
        C.resolve_optimize(cfg)


def test_update_best_model(tmp_path):
    f = tmp_path / "b.yaml"
    with open(f, "w") as h:
        yaml.dump({"fixed_parameters": {"mu": 2e-8}, "optimized_parameters": {},
                   "results": {"log_likelihood": -math.inf, "iteration": None}}, h)
    C.update_best_model(str(f), ["t_1", "r"], [0.0048, 0.5], -10.0, 0)
    C.update_best_model(str(f), ["t_1", "r"], [0.005, 0.6], -11.0, 1)  # worse: kept
    d = yaml.safe_load(open(f))
    assert d["results"] == {"log_likelihood": -10.0, "iteration": 0}
    assert d["optimized_parameters"] == {"t_1": 0.0048 / 2e-8, "r": 0.5 * 2e-8}


def test_write_list(tmp_path):
    from itrails_amd.optimizer import write_list

    f = tmp_path / "h.csv"
    write_list(["n_eval", "t_1", "loglik", "time"], str(f))
    write_list([0, 0.1, -3.5, 1.25], str(f))
    assert open(f).read() == "n_eval,t_1,loglik,time\n0,0.1,-3.5,1.25\n"


# ---------------------------------------------------------------------------------------
# GPU: the commands end to end
# ---------------------------------------------------------------------------------------
def _write_maf(path, obs_blocks, rng):
    """A MAF whose columns encode the given symbols (0..255: A,C,T,G over the 4 species)."""
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
    rng = np.random.default_rng(3)
    blocks = [rng.integers(0, 256, size=int(n)) for n in (300, 1, 57, 800)]
    # runs of a repeated column make the decoded path switch states
    blocks[3][200:500] = 5
    path = tmp_path / "aln.maf"
    _write_maf(path, blocks, rng)
    cfg = _decode_config(tmp_path, settings__n_int_AB=2, settings__n_int_ABC=2,
                         settings__input_maf=str(path))
    cf = tmp_path / "cfg.yaml"
    with open(cf, "w") as h:
        yaml.dump(cfg, h)
    return tmp_path, cf, blocks


def _model_from_setup(s):
    from itrails_amd.model.trans_emiss import trans_emiss_calc

    d = s.params
    return trans_emiss_calc(d["t_A"], d["t_B"], d["t_C"], d["t_2"], d["t_upper"], d["t_out"],
                            d["N_AB"], d["N_ABC"], d["r"], s.n_int_AB, s.n_int_ABC,
                            s.norm_cut_AB, s.norm_cut_ABC)


@pytest.mark.gpu
def test_viterbi_cli_end_to_end(gpu, maf_case):
    from itrails_amd.cli import viterbi_main
    from itrails_amd.tables import build_tables
    from itrails_amd.writers import write_viterbi_csv
    from oracle import hmm_oracle as O

    tmp, cf, blocks = maf_case
    viterbi_main(["--config-file", str(cf), "--output", str(tmp / "v" / "x")])
    cfg = yaml.safe_load(open(cf))
    s = C.resolve_decode(cfg, output_cmd=str(tmp / "chk" / "x"))
    a, b, pi, hidden, _ = _model_from_setup(s)
    obs = np.concatenate(blocks).astype(np.uint16)
    off = np.concatenate([[0], np.cumsum([len(x) for x in blocks])]).astype(np.int64)
    ref_path = O.viterbi(build_tables(a, b, pi), obs, off)
    write_viterbi_csv(str(tmp / "expect.csv"), ref_path.astype(np.uint8), block_off=off)
    assert open(tmp / "v" / "x.viterbi.csv").read() == open(tmp / "expect.csv").read()
    lines = open(tmp / "v" / "x.hidden_states.csv").read().splitlines()
    assert lines[0] == "state_idx,topology,interval_1st_coalescent,interval_2nd_coalescent,shorthand_name"
    assert len(lines) == 1 + len(hidden)
    # a second run into the same prefix writes hidden_states_2.csv (workflow_viterbi.py:637-640)
    viterbi_main(["--config-file", str(cf), "--output", str(tmp / "v" / "x")])
    assert os.path.exists(tmp / "v" / "x.hidden_states_2.csv")


@pytest.mark.gpu
def test_posterior_cli_end_to_end(gpu, maf_case):
    from itrails_amd.cli import posterior_main
    from itrails_amd.tables import build_tables
    from oracle import hmm_oracle as O

    tmp, cf, blocks = maf_case
    posterior_main(["--config-file", str(cf), "--output", str(tmp / "p" / "x")])
    cfg = yaml.safe_load(open(cf))
    s = C.resolve_decode(cfg, output_cmd=str(tmp / "chk" / "x"), kind="posterior")
    a, b, pi, _, _ = _model_from_setup(s)
    obs = np.concatenate(blocks).astype(np.uint16)
    off = np.concatenate([[0], np.cumsum([len(x) for x in blocks])]).astype(np.int64)
    ref = O.posterior(build_tables(a, b, pi), obs, off)
    rows = open(tmp / "p" / "x.posterior.csv").read().splitlines()
    n = a.shape[0]
    assert rows[0] == "alignment_block_idx,position_idx," + ",".join(
        f"prob_state_{j}" for j in range(n))
    got = np.array([[float(v) for v in r.split(",")[2:]] for r in rows[1:]])
    np.testing.assert_allclose(got, ref, rtol=1e-8, atol=1e-300)


@pytest.mark.gpu
def test_optimize_cli_runs(gpu, maf_case):
    from itrails_amd.cli import optimize_main

    tmp, _, _ = maf_case
    cfg = _optimize_config(tmp)
    cfg["settings"].update(n_int_AB=1, n_int_ABC=1, input_maf=str(tmp / "aln.maf"),
                           output_prefix=str(tmp / "o" / "run"))
    cfg["optimized_parameters"] = {"t_1": [240000, 24000, 2400000]}
    # t_upper derived from a fixed t_3 and an optimized N_ABC (workflow_optimize.py:262-290)
    cfg["optimized_parameters"]["N_ABC"] = [50000, 5000, 500000]
    cfg["fixed_parameters"].update(t_2=40000.0, N_AB=50000.0, r=1e-8, t_3=800000.0)
    cf = tmp / "opt.yaml"
    yaml.dump(cfg, open(cf, "w"))
    import itrails_amd.optimizer as OPT

    orig = OPT.optimizer

    def short(**kw):
        return orig(**kw, options={"maxiter": 3, "disp": False})

    OPT.optimizer = short  # optimize_main imports it at call time
    try:
        optimize_main([str(cf)])
    finally:
        OPT.optimizer = orig
    hist = open(tmp / "o" / "run.optimization_history.csv").read().splitlines()
    assert hist[0] == "n_eval,t_1,N_ABC,t_upper,loglik,time"
    assert len(hist) >= 4
    best = yaml.safe_load(open(tmp / "o" / "run.best_model.yaml"))
    lls = [float(r.split(",")[-2]) for r in hist[1:]]
    assert best["results"]["log_likelihood"] == max(lls)
    assert set(best["optimized_parameters"]) == {"t_1", "N_ABC", "t_upper"}


@pytest.mark.gpu
def test_viterbi_cli_config1(gpu, tmp_path):
    """BASELINE config 1 through the drop-in CLI: itrails-viterbi on a synthetic 100 kbp
    (5,5) MAF (gaps and Ns, reference coordinates), viterbi.csv byte-identical to the file
    written from the CPU restatement's paths on the same model and the same parsed input."""
    from itrails_amd.cli import viterbi_main
    from itrails_amd.maf import read_maf
    from itrails_amd.synth import block_lengths, sample_alignment, write_maf
    from itrails_amd.tables import build_tables
    from itrails_amd.writers import write_viterbi_csv
    from oracle import hmm_oracle as O
    from conftest import golden

    g = golden("model_kat_5_5.npz")
    lengths = block_lengths(np.random.default_rng(21), 100_000, 2000.0)
    obs, off, _ = sample_alignment(g["a"], g["b"], g["pi"], lengths, seed=22)
    maf = tmp_path / "chr.maf"
    write_maf(str(maf), obs, off, SP, seed=23)
    cfg = _decode_config(tmp_path, settings__n_int_AB=5, settings__n_int_ABC=5,
                         settings__input_maf=str(maf))
    cfg["settings"]["reference"] = "hg38"
    cf = tmp_path / "cfg.yaml"
    yaml.dump(cfg, open(cf, "w"))
    viterbi_main(["--config-file", str(cf), "--output", str(tmp_path / "v" / "x")])
    s = C.resolve_decode(yaml.safe_load(open(cf)), output_cmd=str(tmp_path / "chk" / "x"))
    a, b, pi, _, _ = _model_from_setup(s)
    robs, roff, coords, _ = read_maf(str(maf), SP, "hg38")
    assert np.array_equal(robs, obs) and np.array_equal(roff, off)
    ref_path = O.viterbi(build_tables(a, b, pi), robs, roff)
    write_viterbi_csv(str(tmp_path / "expect.csv"), ref_path.astype(np.uint8),
                      ref_coordinates=coords, block_off=roff)
    got = open(tmp_path / "v" / "x.viterbi.csv").read()
    assert got == open(tmp_path / "expect.csv").read()
    assert got.count("\n") > len(lengths)  # segments with coordinates, every block present
