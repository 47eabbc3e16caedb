"""Command-line entry points with the reference's surface (pyproject.toml:55-58):

  itrails-optimize  CONFIG.yaml [--input MAF] [--output DIR/PREFIX]       (workflow_optimize.py)
  itrails-viterbi   --config-file F --input MAF --output DIR/PREFIX [...]  (workflow_viterbi.py)
  itrails-posterior --config-file F --input MAF --output DIR/PREFIX [...]  (workflow_posterior.py)
  itrails-int-optimize / itrails-int-viterbi / itrails-int-posterior: the same for the
  introgression model (workflow_int_*.py; pyproject.toml:59-61)

Same options, YAML keys, messages, errors and output files; the model build, the sweeps,
the MAF reader and the CSV writers run on the device path / native library instead of
numba, joblib and Biopython.
"""
from __future__ import annotations

import argparse
import os
import sys

import numpy as np
import yaml

from . import __version__
from .config import (apply_decode_overrides, load_config, resolve_decode,
                     resolve_decode_int, resolve_optimize)


def _decode_parser(kind: str, intro: bool = False) -> argparse.ArgumentParser:
    """workflow_viterbi.py:21-86 (workflow_posterior.py: same options;
    workflow_int_viterbi.py:23-92 adds --t_m, --N_BC and --m)."""
    label = "Viterbi" if kind == "viterbi" else "Posterior"
    prog = f"itrails-int-{kind}" if intro else f"itrails-{kind}"
    p = argparse.ArgumentParser(
        description=f"Run {label} decoding using iTRAILS",
        usage=f"{prog} --config-file CONFIG_FILE --input PATH_MAF --output OUTPUT_PATH "
              "--PARAMETERS")
    p.add_argument("--version", action="version", version=f"%(prog)s {__version__}")
    p.add_argument("--config-file", type=str, required=False, help="Path to the YAML config file.")
    p.add_argument("--input", type=str, required=False, help="Path to the MAF alignment file.")
    p.add_argument("--output", type=str, required=False,
                   help="Path and prefix for output files to be stored. Format: 'directory/prefix'.")
    for name, hlp in (("--mu", "Mutation rate"), ("--t1", "Time parameter t_1"),
                      ("--t_A", "Time to speciation for species A"),
                      ("--t_B", "Time to speciation for species B"),
                      ("--t_C", "Time to speciation for species C"),
                      ("--t2", "Time between first and second speciation"),
                      ("--t3", "Time parameter t_3"), ("--t_upper", "Upper time parameter"),
                      ("--t_out", "Outgroup time parameter"),
                      ("--N_AB", "Effective population size for AB"),
                      ("--N_ABC", "Effective population size for ABC"),
                      ("--r", "Recombination rate")):
        p.add_argument(name, type=float, help=hlp)
    if intro:
        p.add_argument("--t_m", type=float, help="Time parameter t_m")
        p.add_argument("--N_BC", type=float, help="Effective population size for BC")
        p.add_argument("--m", type=float, help="Migration rate between species")
    p.add_argument("--n_cpu", type=int, help="Number of CPUs to use")
    p.add_argument("--species_list", nargs="+", help="List of species names")
    p.add_argument("--reference", type=str, help="Reference to polarize coordinates")
    p.add_argument("--n_int_AB", type=int, help="Number of intervals for AB")
    p.add_argument("--n_int_ABC", type=int, help="Number of intervals for ABC")
    p.add_argument("--cutpoints_AB", nargs="+", type=float, help="Manual cutpoints for AB intervals")
    p.add_argument("--cutpoints_ABC", nargs="+", type=float,
                   help="Manual cutpoints for ABC intervals")
    return p


def _setup_decode(kind: str, argv, intro: bool = False):
    parser = _decode_parser(kind, intro)
    if not argv:
        parser.print_usage()
        sys.exit("Error: No arguments provided. Please provide either a config file, "
                 "command-line parameters, or both.")
    args = parser.parse_args(argv)
    config = {"fixed_parameters": {}, "optimized_parameters": {}, "settings": {}}
    if args.config_file:
        config = load_config(args.config_file)
        for key in ("fixed_parameters", "optimized_parameters", "settings"):
            if config.get(key) is None:
                config[key] = {}
    config = apply_decode_overrides(config, args)
    resolve = resolve_decode_int if intro else resolve_decode
    return resolve(config, args.input, args.output, kind=kind)


def _build_model(s):
    from .model.trans_emiss import trans_emiss_calc

    d = s.params
    print("Calculating transition and emission probability matrices.")
    return trans_emiss_calc(d["t_A"], d["t_B"], d["t_C"], d["t_2"], d["t_upper"], d["t_out"],
                            d["N_AB"], d["N_ABC"], d["r"], s.n_int_AB, s.n_int_ABC,
                            s.norm_cut_AB, s.norm_cut_ABC)


def _build_model_int(s):
    from .model.intro import trans_emiss_calc_introgression

    d = s.params
    print("Calculating transition and emission probability matrices.")
    return trans_emiss_calc_introgression(
        d["t_A"], d["t_B"], d["t_C"], d["t_2"], d["t_upper"], d["t_out"], d["t_m"], d["N_AB"],
        d["N_BC"], d["N_ABC"], d["r"], d["m"], s.n_int_AB, s.n_int_ABC, s.norm_cut_AB,
        s.norm_cut_ABC)


def _read(s):
    from .maf import read_maf

    print("Reading MAF alignment file.")
    obs, off, coords, _ = read_maf(s.maf_path, s.species_list, s.reference)
    return obs, off, coords


def _hidden_states(s, hidden_names, posterior: bool, intro: bool = False):
    from .writers import write_hidden_states_csv, write_hidden_states_csv_int

    f = os.path.join(s.output_dir, f"{s.output_prefix}.hidden_states.csv")
    if os.path.exists(f):
        print(f"Warning: File '{f}' already exists.")
        f = os.path.join(s.output_dir, f"{s.output_prefix}.hidden_states_2.csv")
        print(f"Using an alternative file name: {f}")
    if intro:
        write_hidden_states_csv_int(f, hidden_names, s.abs_cut_AB, s.abs_cut_ABC)
    else:
        write_hidden_states_csv(f, hidden_names, s.abs_cut_AB, s.abs_cut_ABC, posterior)
    print(f"Hidden states written to file {f}.")


def _viterbi(argv, intro: bool) -> None:
    from . import hmm
    from .writers import write_viterbi_csv

    s = _setup_decode("viterbi", sys.argv[1:] if argv is None else argv, intro)
    obs, off, coords = _read(s)
    a, b, pi, hidden_names, _ = (_build_model_int if intro else _build_model)(s)
    _hidden_states(s, hidden_names, posterior=False, intro=intro)
    print("Running viterbi decoding." if intro else "Running viterbi.")
    path = np.zeros(0, dtype=np.uint8)
    if off[-1]:
        model, plan = hmm.Model(a, b, pi), hmm.Plan(off)
        path = hmm._paths(model, plan, obs)
    print("Writing results to file.")
    out = os.path.join(s.output_dir, f"{s.output_prefix}.viterbi.csv")
    write_viterbi_csv(out, path, ref_coordinates=coords, block_off=off)
    print(f"Viterbi decoding complete. Results saved to {out}.")


def _posterior(argv, intro: bool) -> None:
    from . import hmm
    from .writers import write_posterior_csv

    s = _setup_decode("posterior", sys.argv[1:] if argv is None else argv, intro)
    obs, off, coords = _read(s)
    a, b, pi, hidden_names, _ = (_build_model_int if intro else _build_model)(s)
    _hidden_states(s, hidden_names, posterior=True, intro=intro)
    print("Running posterior decoding.")
    n = a.shape[0]
    post = np.zeros((0, n))
    if off[-1]:
        model, plan = hmm.Model(a, b, pi), hmm.Plan(off)
        post = hmm._posteriors(model, plan, obs)
    print("Writing results to file.")
    out = os.path.join(s.output_dir, f"{s.output_prefix}.posterior.csv")
    write_posterior_csv(out, post, ref_coordinates=coords, block_off=off, threads=s.n_cpu)
    print(f"Posterior decoding complete. Results saved to {out}.")


def viterbi_main(argv=None) -> None:
    """itrails-viterbi (workflow_viterbi.py:19-745)."""
    _viterbi(argv, intro=False)


def posterior_main(argv=None) -> None:
    """itrails-posterior (workflow_posterior.py:19-717)."""
    _posterior(argv, intro=False)


def int_viterbi_main(argv=None) -> None:
    """itrails-int-viterbi (workflow_int_viterbi.py:21-776)."""
    _viterbi(argv, intro=True)


def int_posterior_main(argv=None) -> None:
    """itrails-int-posterior (workflow_int_posterior.py:21-743)."""
    _posterior(argv, intro=True)


def _optimize(argv, intro: bool) -> None:
    from .maf import maf_parser
    from .optimizer import optimizer, optimizer_introgression

    parser = argparse.ArgumentParser(
        description=("Optimize workflow with introgression using TRAILS" if intro
                     else "Optimize workflow using TRAILS"),
        usage=("itrails-optimize <config.yaml> --input PATH_TO_MAF --output OUTPUT_PATH" if intro
               else "itrails-optimize <config.yaml> --output OUTPUT_PATH | itrails-optimize "
                    "example --output OUTPUT_PATH"))
    parser.add_argument("--version", action="version", version=f"%(prog)s {__version__}")
    parser.add_argument("config_file", type=str, help="Path to the YAML config file.")
    parser.add_argument("--input", type=str, required=False, help="Path to the MAF alignment file.")
    parser.add_argument("--output", type=str, required=False,
                        help="Path and prefix for output files to be stored. Format: 'directory/prefix'.")
    args = parser.parse_args(sys.argv[1:] if argv is None else argv)
    config = load_config(args.config_file)
    s = resolve_optimize(config, args.input, args.output, intro=intro)
    sep = "_" if intro else "."  # the introgression workflow names its files prefix_*.
    with open(os.path.join(s.output_dir, f"{s.output_prefix}{sep}starting_params.yaml"), "w") as f:
        yaml.dump(s.starting_params, f, default_flow_style=False)
    best = os.path.join(s.output_dir, f"{s.output_prefix}{sep}best_model.yaml")
    with open(best, "w") as f:
        yaml.dump(s.best_model, f)
    V_lst = maf_parser(s.maf_path, s.species_list)
    if V_lst is None:
        raise ValueError("Error reading MAF alignment file.")
    print("Running optimization...")
    run = optimizer_introgression if intro else optimizer
    run(optim_variables=s.optim_variables, optim_list=s.optim_list, bounds=s.bounds,
        fixed_params=s.fixed, V_lst=V_lst, res_name=s.output, case=s.case,
        method=s.method, header=True)
    hist = os.path.join(s.output_dir, f"{s.output_prefix}{sep}optimization_history.csv")
    print(f"Optimization complete. Results saved to {hist}.\n Best model saved to {best}.")


def optimize_main(argv=None) -> None:
    """itrails-optimize (workflow_optimize.py:17-489)."""
    _optimize(argv, intro=False)


def int_optimize_main(argv=None) -> None:
    """itrails-int-optimize (workflow_int_optimize.py:17-474)."""
    _optimize(argv, intro=True)


def main(argv=None) -> None:
    """`python -m itrails_amd {optimize|viterbi|posterior|int-optimize|int-viterbi|
    int-posterior} ...`"""
    argv = sys.argv[1:] if argv is None else argv
    cmds = {"optimize": optimize_main, "viterbi": viterbi_main, "posterior": posterior_main,
            "int-optimize": int_optimize_main, "int-viterbi": int_viterbi_main,
            "int-posterior": int_posterior_main}
    if not argv or argv[0] not in cmds:
        sys.exit("usage: python -m itrails_amd {optimize|viterbi|posterior|int-optimize|"
                 "int-viterbi|int-posterior} ...")
    cmds[argv[0]](argv[1:])
