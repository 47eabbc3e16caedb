"""Command-line entry points with the reference's surface (pyproject.toml:55-58):

  itrails-optimize  CONFIG.yaml [--input MAF] [--output DIR/PREFIX]       (workflow_optimize.py)
  itrails-viterbi   --config-file F --input MAF --output DIR/PREFIX [...]  (workflow_viterbi.py)
  itrails-posterior --config-file F --input MAF --output DIR/PREFIX [...]  (workflow_posterior.py)

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
                     resolve_optimize)


def _decode_parser(kind: str) -> argparse.ArgumentParser:
    """workflow_viterbi.py:21-86 (workflow_posterior.py: same options)."""
    label = "Viterbi" if kind == "viterbi" else "Posterior"
    p = argparse.ArgumentParser(
        description=f"Run {label} decoding using iTRAILS",
        usage=f"itrails-{kind} --config-file CONFIG_FILE --input PATH_MAF --output OUTPUT_PATH "
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
    p.add_argument("--n_cpu", type=int, help="Number of CPUs to use")
    p.add_argument("--species_list", nargs="+", help="List of species names")
    p.add_argument("--reference", type=str, help="Reference to polarize coordinates")
    p.add_argument("--n_int_AB", type=int, help="Number of intervals for AB")
    p.add_argument("--n_int_ABC", type=int, help="Number of intervals for ABC")
    p.add_argument("--cutpoints_AB", nargs="+", type=float, help="Manual cutpoints for AB intervals")
    p.add_argument("--cutpoints_ABC", nargs="+", type=float,
                   help="Manual cutpoints for ABC intervals")
    return p


def _setup_decode(kind: str, argv):
    parser = _decode_parser(kind)
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
    return resolve_decode(config, args.input, args.output, kind=kind)


def _build_model(s):
    from .model.trans_emiss import trans_emiss_calc

    d = s.params
    print("Calculating transition and emission probability matrices.")
    return trans_emiss_calc(d["t_A"], d["t_B"], d["t_C"], d["t_2"], d["t_upper"], d["t_out"],
                            d["N_AB"], d["N_ABC"], d["r"], s.n_int_AB, s.n_int_ABC,
                            s.norm_cut_AB, s.norm_cut_ABC)


def _read(s):
    from .maf import read_maf

    print("Reading MAF alignment file.")
    obs, off, coords, _ = read_maf(s.maf_path, s.species_list, s.reference)
    return obs, off, coords


def _hidden_states(s, hidden_names, posterior: bool):
    from .writers import write_hidden_states_csv

    f = os.path.join(s.output_dir, f"{s.output_prefix}.hidden_states.csv")
    if os.path.exists(f):
        print(f"Warning: File '{f}' already exists.")
        f = os.path.join(s.output_dir, f"{s.output_prefix}.hidden_states_2.csv")
        print(f"Using an alternative file name: {f}")
    write_hidden_states_csv(f, hidden_names, s.abs_cut_AB, s.abs_cut_ABC, posterior)
    print(f"Hidden states written to file {f}.")


def viterbi_main(argv=None) -> None:
    """itrails-viterbi (workflow_viterbi.py:19-745)."""
    from . import hmm
    from .writers import write_viterbi_csv

    s = _setup_decode("viterbi", sys.argv[1:] if argv is None else argv)
    obs, off, coords = _read(s)
    a, b, pi, hidden_names, _ = _build_model(s)
    _hidden_states(s, hidden_names, posterior=False)
    print("Running viterbi.")
    path = np.zeros(0, dtype=np.uint8)
    if off[-1]:
        model, plan = hmm.Model(a, b, pi), hmm.Plan(off)
        path = hmm._paths(model, plan, obs)
    print("Writing results to file.")
    out = os.path.join(s.output_dir, f"{s.output_prefix}.viterbi.csv")
    write_viterbi_csv(out, path, ref_coordinates=coords, block_off=off)
    print(f"Viterbi decoding complete. Results saved to {out}.")


def posterior_main(argv=None) -> None:
    """itrails-posterior (workflow_posterior.py:19-717)."""
    from . import hmm
    from .writers import write_posterior_csv

    s = _setup_decode("posterior", sys.argv[1:] if argv is None else argv)
    obs, off, coords = _read(s)
    a, b, pi, hidden_names, _ = _build_model(s)
    _hidden_states(s, hidden_names, posterior=True)
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


def optimize_main(argv=None) -> None:
    """itrails-optimize (workflow_optimize.py:17-489)."""
    from .maf import maf_parser
    from .optimizer import optimizer

    parser = argparse.ArgumentParser(
        description="Optimize workflow using TRAILS",
        usage="itrails-optimize <config.yaml> --output OUTPUT_PATH | itrails-optimize example "
              "--output OUTPUT_PATH")
    parser.add_argument("--version", action="version", version=f"%(prog)s {__version__}")
    parser.add_argument("config_file", type=str, help="Path to the YAML config file.")
    parser.add_argument("--input", type=str, required=False, help="Path to the MAF alignment file.")
    parser.add_argument("--output", type=str, required=False,
                        help="Path and prefix for output files to be stored. Format: 'directory/prefix'.")
    args = parser.parse_args(sys.argv[1:] if argv is None else argv)
    config = load_config(args.config_file)
    s = resolve_optimize(config, args.input, args.output)
    with open(os.path.join(s.output_dir, f"{s.output_prefix}.starting_params.yaml"), "w") as f:
        yaml.dump(s.starting_params, f, default_flow_style=False)
    best = os.path.join(s.output_dir, f"{s.output_prefix}.best_model.yaml")
    with open(best, "w") as f:
        yaml.dump(s.best_model, f)
    V_lst = maf_parser(s.maf_path, s.species_list)
    if V_lst is None:
        raise ValueError("Error reading MAF alignment file.")
    print("Running optimization...")
    optimizer(optim_variables=s.optim_variables, optim_list=s.optim_list, bounds=s.bounds,
              fixed_params=s.fixed, V_lst=V_lst, res_name=s.output, case=s.case,
              method=s.method, header=True)
    hist = os.path.join(s.output_dir, f"{s.output_prefix}.optimization_history.csv")
    print(f"Optimization complete. Results saved to {hist}.\n Best model saved to {best}.")


def main(argv=None) -> None:
    """`python -m itrails_amd {optimize|viterbi|posterior} ...`"""
    argv = sys.argv[1:] if argv is None else argv
    cmds = {"optimize": optimize_main, "viterbi": viterbi_main, "posterior": posterior_main}
    if not argv or argv[0] not in cmds:
        sys.exit("usage: python -m itrails_amd {optimize|viterbi|posterior} ...")
    cmds[argv[0]](argv[1:])
