"""YAML / command-line parameter resolution of the itrails-* entry points.

Restates, in the reference's order and with its messages and errors, how the decode CLIs
(workflow_viterbi.py:88-611, workflow_posterior.py: same lines) and the optimizer CLI
(workflow_optimize.py:46-470) turn a config file plus overrides into the internal
parameter dictionary (times and population sizes multiplied by mu, r divided by mu), the
time-parameter "case", the cutpoints and the optimizer's start vector and bounds.  The
per-evaluation derivation of t_A/t_B/t_C/t_out from the case is shared with the
optimizer loop (optimizer.py:419-541).

Quirks kept on purpose: a decode run derives t_upper from t_3 unless
t_upper is an *optimized* parameter (workflow_viterbi.py:361,403 — the fixed branch is
unreachable); decode runs use the given or normalised cutpoints, the optimizer always the
"standard" ones.
"""
from __future__ import annotations

import math
import os
import sys
from typing import Dict, List, Optional, Tuple

import yaml

from .model.emissions import cutpoints_AB, cutpoints_ABC

TIME_COMBINATIONS = {
    frozenset(["t_A", "t_B", "t_C"]),
    frozenset(["t_1", "t_A"]),
    frozenset(["t_1", "t_B"]),
    frozenset(["t_1", "t_C"]),
    frozenset(["t_A", "t_B"]),
    frozenset(["t_A", "t_C"]),
    frozenset(["t_B", "t_C"]),
    frozenset(["t_1"]),
}
CORE_PARAMS = ["t_2", "N_ABC", "N_AB", "r"]


# ---------------------------------------------------------------------------------------
# YAML helpers (yaml_helpers.py:7-118)
# ---------------------------------------------------------------------------------------
class FlowSeq(list):
    """A list dumped in YAML flow style ([a, b, c])."""


def _flow_seq(dumper, data):
    return dumper.represent_sequence("tag:yaml.org,2002:seq", data, flow_style=True)


yaml.add_representer(FlowSeq, _flow_seq)


def load_config(path: str):
    """yaml_helpers.py:35-53: parse the file; on any error print it and exit(1)."""
    try:
        with open(path, "r") as f:
            return yaml.safe_load(f)
    except Exception as e:  # the reference's behaviour: report and exit
        print(f"Error loading config file: {e}", file=sys.stderr)
        sys.exit(1)


def update_best_model(best_model_yaml: str, optim_variables, values, loglik: float,
                      iteration: int) -> None:
    """yaml_helpers.py:56-118: rewrite best_model.yaml when `loglik` beats the stored one,
    with the optimized values converted back to user units (r * mu, others / mu)."""
    if not os.path.exists(best_model_yaml):
        raise FileNotFoundError(f"Best model file not found: {best_model_yaml}")
    with open(best_model_yaml, "r") as f:
        try:
            data = yaml.safe_load(f)
        except yaml.YAMLError as e:
            print(f"Error loading best model file: {e}")
            sys.exit(1)
    mu = float(data["fixed_parameters"]["mu"])
    prev = data["results"]["log_likelihood"]
    if prev is not None and not loglik > prev:
        return
    data["optimized_parameters"] = {
        v: (float(values[i]) * mu if v == "r" else float(values[i]) / mu)
        for i, v in enumerate(optim_variables)}
    data["results"]["log_likelihood"] = loglik
    data["results"]["iteration"] = iteration
    with open(best_model_yaml, "w") as f:
        yaml.dump(data, f)


# ---------------------------------------------------------------------------------------
# CPU count (ncpu.py:1-34)
# ---------------------------------------------------------------------------------------
def available_cpus() -> int:
    return int(os.environ.get("SLURM_JOB_CPUS_PER_NODE", os.cpu_count() or 1))


def update_n_cpu(requested) -> int:
    """ncpu.py:8-34: min(requested, available), exported to the numerical libraries'
    thread-count variables.  The GPU path does not fan out over host processes; the count
    only sizes host-side helpers (MAF reader, CSV writers)."""
    avail = available_cpus()
    try:
        req = int(requested)
    except (TypeError, ValueError):
        req = avail
    n = min(req, avail)
    for var in ("OMP_NUM_THREADS", "MKL_NUM_THREADS", "NUMEXPR_NUM_THREADS",
                "RAYON_NUM_THREADS", "RAY_NUM_THREADS"):
        os.environ[var] = str(n)
    print(f"Using {n} CPU cores (requested: {req}, available: {avail}).")
    return n


# ---------------------------------------------------------------------------------------
# shared pieces
# ---------------------------------------------------------------------------------------
def resolve_io(input_cmd: Optional[str], output_cmd: Optional[str], input_config,
               output_config) -> Tuple[str, str]:
    """workflow_viterbi.py:155-199: command line wins over the config (with a warning);
    missing input or output is a ValueError.  -> (maf_path, output 'dir/prefix')."""
    if input_cmd and input_config:
        print(f"Warning: MAF alignment file specified in both config file ({input_config}) "
              f"and command-line ({input_cmd}). Using command-line input.")
        maf_path = input_cmd
    elif input_cmd or input_config:
        maf_path = input_cmd or input_config
        print(f"Using MAF alignment file: {maf_path}")
    else:
        raise ValueError("Error: MAF alignment file not specified in config file or command-line.")
    if output_cmd and output_config:
        print(f"Warning: Output file specified in both config file ({output_config}) and "
              f"command-line ({output_cmd}). Using command-line output.")
        out = output_cmd
    elif output_cmd or output_config:
        out = output_cmd or output_config
    else:
        raise ValueError("Error: Output file not specified in config file or command-line.")
    return maf_path, out


def derive_times(d: Dict, case: frozenset, cut_abc_last: float) -> Dict:
    """The case table of workflow_viterbi.py:433-568 / optimizer.py:419-541, on internal
    (mu-scaled) values: completes t_A, t_B, t_C and t_out (unless t_out is fixed) and drops
    t_1.  `cut_abc_last` is the last finite normalised ABC cutpoint."""
    d = dict(d)
    fixed_out = "t_out" in d

    def outgroup(base):  # summed left to right, as the reference writes it
        return base + cut_abc_last * d["N_ABC"] + d["t_upper"] + 2 * d["N_ABC"]

    if "t_1" in case:
        t1 = d["t_1"]
        if case == frozenset(["t_1", "t_A"]):
            d["t_B"], d["t_C"] = t1, t1 + d["t_2"]
        elif case == frozenset(["t_1", "t_B"]):
            d["t_A"], d["t_C"] = t1, t1 + d["t_2"]
        elif case == frozenset(["t_1", "t_C"]):
            d["t_A"], d["t_B"] = t1, t1
        else:  # {t_1}
            d["t_A"], d["t_B"], d["t_C"] = t1, t1, t1 + d["t_2"]
        if not fixed_out:
            d["t_out"] = outgroup(t1 + d["t_2"])
        d.pop("t_1")
        return d
    if case == frozenset(["t_A", "t_B"]):
        d["t_C"] = (d["t_A"] + d["t_B"]) / 2 + d["t_2"]
    elif case == frozenset(["t_A", "t_C"]):
        d["t_B"] = (d["t_A"] + d["t_C"] - d["t_2"]) / 2
    elif case == frozenset(["t_B", "t_C"]):
        d["t_A"] = (d["t_B"] + d["t_C"] - d["t_2"]) / 2
    if not fixed_out:
        d["t_out"] = outgroup((((d["t_A"] + d["t_B"]) / 2 + d["t_2"]) + d["t_C"]) / 2)
    return d


def derive_times_int(d: Dict, case: frozenset, cut_abc_last: float) -> Dict:
    """The introgression model's case table (int_optimizer.py:404-529,
    workflow_int_viterbi.py:456-586): B and C split from the lineage t_m before the first
    speciation, so t_B = t_C = t_1 - t_m and the outgroup base averages t_B + t_m and
    t_C + t_m + t_2."""
    d = dict(d)
    fixed_out = "t_out" in d

    def outgroup(base):
        return base + cut_abc_last * d["N_ABC"] + d["t_upper"] + 2 * d["N_ABC"]

    def averaged():  # summed left to right, as the reference writes it
        return (((d["t_A"] + (d["t_B"] + d["t_m"])) / 2 + d["t_2"])
                + (d["t_C"] + d["t_m"] + d["t_2"]) / 2)

    if "t_1" in case:
        t1, tm = d["t_1"], d["t_m"]
        if case == frozenset(["t_1", "t_A"]):
            d["t_B"] = d["t_C"] = t1 - tm
        elif case == frozenset(["t_1", "t_B"]):
            d["t_A"], d["t_C"] = t1, t1 - tm
        elif case == frozenset(["t_1", "t_C"]):
            d["t_A"], d["t_B"] = t1, t1 - tm
        else:  # {t_1}
            d["t_A"] = t1
            d["t_B"] = d["t_C"] = t1 - tm
        if not fixed_out:
            d["t_out"] = outgroup(t1 + d["t_2"])
        d.pop("t_1")
        return d
    if case == frozenset(["t_A", "t_B"]):
        d["t_C"] = (d["t_B"] + d["t_A"] + d["t_m"]) / 2
    elif case == frozenset(["t_A", "t_C"]):
        d["t_B"] = (d["t_C"] + d["t_A"] + d["t_m"]) / 2
    elif case == frozenset(["t_B", "t_C"]):
        d["t_A"] = (d["t_C"] + d["t_B"] + d["t_m"]) / 2
    if not fixed_out:
        d["t_out"] = outgroup(averaged())
    return d


def _time_values(fixed: Dict, optimized: Dict, found: set, with_bounds: bool):
    """process_parameter of workflow_viterbi.py:276-289 / workflow_optimize.py:149-169."""
    out = {}
    for p in ("t_1", "t_A", "t_B", "t_C"):
        if p in fixed and p in optimized:
            raise ValueError(f"Parameter '{p}' cannot be both fixed and optimized.")
        if p in fixed:
            found.add(p)
            out[p] = (fixed[p], None, None, True)
        elif p in optimized:
            found.add(p)
            v = optimized[p]
            out[p] = (v[0], v[1], v[2], False) if with_bounds else (v, None, None, False)
    return out


# ---------------------------------------------------------------------------------------
# decode CLIs (itrails-viterbi / itrails-posterior)
# ---------------------------------------------------------------------------------------
class DecodeSetup:
    """Everything a decode run needs after validation."""

    def __init__(self):
        self.maf_path = ""
        self.output = ""
        self.output_dir = ""
        self.output_prefix = ""
        self.species_list: List[str] = []
        self.reference: Optional[str] = None
        self.params: Dict = {}       # internal units: t_A t_B t_C t_2 t_upper t_out N_AB N_ABC r
        self.n_int_AB = 0
        self.n_int_ABC = 0
        self.norm_cut_AB: List[float] = []
        self.norm_cut_ABC: List[float] = []
        self.abs_cut_AB: List[float] = []
        self.abs_cut_ABC: List[float] = []
        self.mu = 0.0
        self.n_cpu = 1


def apply_decode_overrides(config: Dict, args) -> Dict:
    """workflow_viterbi.py:88-153 (workflow_int_viterbi.py:94-160 adds t_m, N_BC and m):
    command-line values replace the config's and move a parameter from
    optimized_parameters to fixed_parameters."""
    if args.mu is not None:
        config["fixed_parameters"]["mu"] = args.mu
    elif "mu" not in config["fixed_parameters"]:
        raise ValueError("Error: mu must be specified either in config file or via --mu")
    moved = {"t_1": args.t1, "t_A": args.t_A, "t_B": args.t_B, "t_C": args.t_C,
             "t_2": args.t2, "t_3": args.t3, "t_upper": args.t_upper, "t_out": args.t_out,
             "N_AB": args.N_AB, "N_ABC": args.N_ABC, "r": args.r}
    for p in ("t_m", "N_BC", "m"):  # introgression CLIs only
        if hasattr(args, p):
            moved[p] = getattr(args, p)
    for p, v in moved.items():
        if v is not None:
            config["optimized_parameters"].pop(p, None)
            config["fixed_parameters"][p] = v
    for key in ("n_cpu", "species_list", "reference", "n_int_AB", "n_int_ABC",
                "cutpoints_AB", "cutpoints_ABC"):
        v = getattr(args, key)
        if v is not None:
            config["settings"][key] = v
    return config


def resolve_decode(config: Dict, input_cmd=None, output_cmd=None, kind="viterbi",
                   verbose=True) -> DecodeSetup:
    """workflow_viterbi.py:155-611 (kind "viterbi") / workflow_posterior.py (kind
    "posterior"): validate and convert the parameters; creates the output directory."""
    s = DecodeSetup()
    settings = config["settings"]
    s.maf_path, s.output = resolve_io(input_cmd, output_cmd, settings.get("input_maf"),
                                      settings.get("output_prefix"))
    s.output_dir, s.output_prefix = os.path.split(s.output)
    os.makedirs(s.output_dir, exist_ok=True)
    print(f"Results will be saved to: {s.output_dir} as '{s.output_prefix}.{kind}.csv'.")
    requested = settings.get("n_cpu")
    s.n_cpu = update_n_cpu(requested)
    if requested is None:
        print(f"No CPU count specified in config; using default {s.n_cpu} cores.")

    cut_AB, cut_ABC = settings.get("cutpoints_AB"), settings.get("cutpoints_ABC")
    n_int_AB, n_int_ABC = settings.get("n_int_AB"), settings.get("n_int_ABC")
    if not n_int_AB and not cut_AB:
        raise ValueError("Error: n_int_AB must be specified in the config file for automatic "
                         "cutpoints, n_int_AB and cutpoints_AB must be specified in the config "
                         "file for manual cutpoints.")
    if not n_int_ABC and not cut_ABC:
        raise ValueError("Error: n_int_ABC must be specified in the config file for automatic "
                         "cutpoints, n_int_ABC and cutpoints_ABC must be specified in the "
                         "config file for manual cutpoints.")
    if (cut_AB and n_int_AB) and len(cut_AB) != n_int_AB + 1:
        raise ValueError("Error: cutpoints_AB must have n_int_AB + 1 values, check the config file.")
    if (cut_ABC and n_int_ABC) and len(cut_ABC) != n_int_ABC:
        raise ValueError("Error: cutpoints_ABC must have n_int_ABC values, check the config file.")

    fixed, optimized = config["fixed_parameters"], config["optimized_parameters"]
    s.species_list = settings["species_list"]
    s.reference = settings.get("reference")
    mu = float(fixed["mu"])
    s.mu = mu
    d: Dict = {}
    if not (isinstance(n_int_AB, int) and n_int_AB > 0):
        raise ValueError("n_int_AB must be a positive integer")
    if not (isinstance(n_int_ABC, int) and n_int_ABC > 0):
        raise ValueError("n_int_ABC must be a positive integer")
    if mu <= 0:
        raise ValueError("mu must be a positive float or int.")
    s.n_int_AB, s.n_int_ABC = n_int_AB, n_int_ABC

    optim_vars: List[str] = []
    optim_vals: List = []
    pre: Dict = {}
    for p in CORE_PARAMS:
        if p in fixed and p in optimized:
            raise ValueError(f"Parameter '{p}' cannot be both fixed and optimized.")
        if p in fixed:
            pre[p] = float(fixed[p])
            d[p] = fixed[p]
        elif p in optimized:
            pre[p] = float(optimized[p])
            optim_vars.append(p)
            optim_vals.append(optimized[p])
        else:
            raise ValueError("Parameters 't_2', 'N_ABC', 'N_AB' and 'r' must be present in "
                             "optimized or fixed parameters.")
    found: set = set()
    tv = _time_values(fixed, optimized, found, with_bounds=False)
    if frozenset(found) not in TIME_COMBINATIONS:
        raise ValueError(f"Invalid combination of time values: {found}, check possible "
                         "combinations in the documentation.")
    for p in ("t_1", "t_A", "t_B", "t_C"):
        if p in found:
            v, _, _, is_fixed = tv[p]
            if is_fixed:
                d[p] = v
            else:
                optim_vars.append(p)
                optim_vals.append(v)
    pre_t_A = float(tv["t_A"][0]) if "t_A" in found else float(tv["t_1"][0])
    case = frozenset(found)
    if "t_out" in fixed:
        d["t_out"] = fixed["t_out"]
    elif "t_out" in optimized:
        raise ValueError("Parameter 't_out' has to be fixed.")

    if cut_AB is None:
        abs_cut_AB = [pre_t_A + x for x in cutpoints_AB(n_int_AB, pre["t_2"], 1 / pre["N_AB"])]
        norm_cut_AB = [(x - pre_t_A) / pre["N_ABC"] for x in abs_cut_AB]
    else:
        abs_cut_AB = [float(x) for x in cut_AB]
        norm_cut_AB = [(float(x) - pre_t_A) / pre["N_ABC"] for x in cut_AB]
    if cut_ABC is None:
        norm_cut_ABC = list(cutpoints_ABC(n_int_ABC, 1))
        abs_cut_ABC = [float(x) * pre["N_ABC"] + pre_t_A + pre["t_2"] for x in norm_cut_ABC]
    else:
        abs_cut_ABC = [float(x) for x in cut_ABC]
        norm_cut_ABC = [(x - pre_t_A - pre["t_2"]) / pre["N_ABC"] for x in abs_cut_ABC]
        norm_cut_ABC.append(float("inf"))

    # t_upper (workflow_viterbi.py:360-404): derived from t_3 unless optimized
    if "t_upper" not in optimized:
        print("Warning: 't_upper' not found in parameter definition. Calculating from 't_3' "
              "and 'N_ABC'.")
        if "N_ABC" in optimized or "N_ABC" in fixed:
            n_abc = optimized["N_ABC"] if "N_ABC" in optimized else fixed["N_ABC"]
            t3 = optimized.get("t_3", fixed.get("t_3"))
            if t3 is None:
                raise ValueError("'t_3' not found in parameter definition.")
            optim_vars.append("t_upper")
            optim_vals.append(t3 - norm_cut_ABC[-2] * n_abc)
        else:
            raise ValueError("'N_ABC' not found in parameter definition.")
    else:
        optim_vars.append("t_upper")
        optim_vals.append(optimized["t_upper"])

    for i, p in enumerate(optim_vars):
        if p in fixed:
            raise ValueError(f"Parameter '{p}' cannot be present in both fixed and "
                             "optimized parameters.")
        v = float(optim_vals[i])
        if v <= 0:
            raise ValueError(f"Value for '{p}' must be a positive number.")
        optim_vals[i] = v / mu if p == "r" else v * mu
    for p in list(d):
        d[p] = float(d[p]) / mu if p == "r" else float(d[p]) * mu
    for i, p in enumerate(optim_vars):
        d[p] = optim_vals[i]
    if d["t_upper"] < 0:
        raise ValueError("Parameter 't_upper' must be a positive number. "
                         f"Given/calculated value: {d['t_upper']}")
    d = derive_times(d, case, norm_cut_ABC[-2])

    # cutpoint ranges (workflow_viterbi.py:570-599)
    lo, hi = pre_t_A, pre_t_A + pre["t_2"]
    early = abs_cut_AB[0] < lo and not math.isclose(abs_cut_ABC[0], lo, rel_tol=1e-9, abs_tol=1e-12)
    late = abs_cut_AB[-1] > hi and not math.isclose(abs_cut_ABC[-1], hi, rel_tol=1e-9, abs_tol=1e-12)
    if early or late:
        raise ValueError("cutpoints_AB must lie within [t_A, t_A + t_2]."
                         f"Given cutpoints_AB: {abs_cut_AB}, t_A: {lo}, t_A + t_2: {hi}.")
    lo, hi = pre_t_A + pre["t_2"], d["t_out"] / mu
    early = abs_cut_ABC[0] < lo and not math.isclose(abs_cut_ABC[0], lo, rel_tol=1e-9, abs_tol=1e-12)
    late = abs_cut_ABC[-2] > hi and not math.isclose(abs_cut_ABC[-2], hi, rel_tol=1e-9, abs_tol=1e-12)
    if early or late:
        raise ValueError("cutpoints_ABC must lie within [t_A + t_2, t_out]."
                         f"Given cutpoints_ABC: {abs_cut_ABC}, t_A + t_2: {lo}, t_out: {hi}.")
    if verbose:
        print("Parameters validated:")
        print(f"Cutpoints AB: {abs_cut_AB}")
        print(f"Cutpoints ABC: {abs_cut_ABC}")
        print(f"n_int_AB: {n_int_AB}")
        print(f"n_int_ABC: {n_int_ABC}")
        for k, v in d.items():
            print(f"{k}: {v * mu if k == 'r' else v / mu}")
    s.params = d
    s.norm_cut_AB, s.norm_cut_ABC = norm_cut_AB, norm_cut_ABC
    s.abs_cut_AB, s.abs_cut_ABC = abs_cut_AB, abs_cut_ABC
    return s


INT_CORE_PARAMS = ["t_2", "N_ABC", "N_AB", "N_BC", "r", "t_m", "m"]
_INT_MISSING = ("Parameters 't_2', 'N_ABC', 'N_AB', 'N_BC, 't_m', 'm' and 'r' must be present "
                "in optimized or fixed parameters.")


def resolve_decode_int(config: Dict, input_cmd=None, output_cmd=None, kind="viterbi",
                       verbose=True) -> DecodeSetup:
    """itrails-int-viterbi / itrails-int-posterior parameter resolution
    (workflow_int_viterbi.py:162-612; workflow_int_posterior.py: same lines).  Differs from
    the plain model's: t_m, N_BC and m are mandatory; settings.proportional makes t_m a
    fraction of t_1 ({t_1} case only); the positivity checks are commented out in the
    reference, so none are made here; every parameter except r — the admixture
    proportion m included — is multiplied by mu (workflow_int_viterbi.py:446-451, kept as
    the reference computes it)."""
    s = DecodeSetup()
    settings = config["settings"]
    s.maf_path, s.output = resolve_io(input_cmd, output_cmd, settings.get("input_maf"),
                                      settings.get("output_prefix"))
    s.output_dir, s.output_prefix = os.path.split(s.output)
    os.makedirs(s.output_dir, exist_ok=True)
    print(f"Results will be saved to: {s.output_dir} as '{s.output_prefix}.{kind}.csv'.")
    requested = settings.get("n_cpu")
    s.n_cpu = update_n_cpu(requested)
    if requested is None:
        print(f"No CPU count specified in config; using default {s.n_cpu} cores.")

    cut_AB, cut_ABC = settings.get("cutpoints_AB"), settings.get("cutpoints_ABC")
    n_int_AB, n_int_ABC = settings.get("n_int_AB"), settings.get("n_int_ABC")
    proportional_tm = settings.get("proportional")
    if not n_int_AB and not cut_AB:
        raise ValueError("Error: n_int_AB must be specified in the config file for automatic "
                         "cutpoints, n_int_AB and cutpoints_AB must be specified in the config "
                         "file for manual cutpoints.")
    if not n_int_ABC and not cut_ABC:
        raise ValueError("Error: n_int_ABC must be specified in the config file for automatic "
                         "cutpoints, n_int_ABC and cutpoints_ABC must be specified in the "
                         "config file for manual cutpoints.")
    if (cut_AB and n_int_AB) and len(cut_AB) != n_int_AB + 1:
        raise ValueError("Error: cutpoints_AB must have n_int_AB + 1 values, check the config file.")
    if (cut_ABC and n_int_ABC) and len(cut_ABC) != n_int_ABC:
        raise ValueError("Error: cutpoints_ABC must have n_int_ABC values, check the config file.")

    fixed, optimized = config["fixed_parameters"], config["optimized_parameters"]
    s.species_list = settings["species_list"]
    s.reference = settings.get("reference")
    mu = float(fixed["mu"])
    s.mu = mu
    d: Dict = {}
    if not (isinstance(n_int_AB, int) and n_int_AB > 0):
        raise ValueError("n_int_AB must be a positive integer")
    d["n_int_AB"] = n_int_AB
    if not (isinstance(n_int_ABC, int) and n_int_ABC > 0):
        raise ValueError("n_int_ABC must be a positive integer")
    d["n_int_ABC"] = n_int_ABC
    if mu <= 0:
        raise ValueError("mu must be a positive float or int.")
    s.n_int_AB, s.n_int_ABC = n_int_AB, n_int_ABC

    optim_vars: List[str] = []
    optim_vals: List = []
    pre: Dict = {}
    for p in INT_CORE_PARAMS:
        if p in fixed and p in optimized:
            raise ValueError(f"Parameter '{p}' cannot be both fixed and optimized.")
        if p in fixed:
            pre[p] = fixed[p]
            d[p] = fixed[p]
        elif p in optimized:
            pre[p] = optimized[p]
            optim_vars.append(p)
            optim_vals.append(optimized[p])
        else:
            raise ValueError(_INT_MISSING)
    found: set = set()
    tv = _time_values(fixed, optimized, found, with_bounds=False)
    if frozenset(found) not in TIME_COMBINATIONS:
        raise ValueError(f"Invalid combination of time values: {found}, check possible "
                         "combinations in the documentation.")
    for p in ("t_1", "t_A", "t_B", "t_C"):
        if p in found:
            v, _, _, is_fixed = tv[p]
            if is_fixed:
                d[p] = v
            else:
                optim_vars.append(p)
                optim_vals.append(v)
    pre_t_A = tv["t_A"][0] if "t_A" in found else tv["t_1"][0]
    case = frozenset(found)
    if "t_out" in fixed:
        d["t_out"] = fixed["t_out"]
    elif "t_out" in optimized:
        raise ValueError("Parameter 't_out' has to be fixed.")

    if cut_AB is None:
        abs_cut_AB = [pre_t_A + x for x in cutpoints_AB(n_int_AB, pre["t_2"], 1 / pre["N_AB"])]
        norm_cut_AB = [(x - pre_t_A) / pre["N_ABC"] for x in abs_cut_AB]
    else:
        abs_cut_AB = [float(x) for x in cut_AB]
        norm_cut_AB = [(float(x) - pre_t_A) / pre["N_ABC"] for x in cut_AB]
    if cut_ABC is None:
        norm_cut_ABC = list(cutpoints_ABC(n_int_ABC, 1))
        abs_cut_ABC = [float(x) * pre["N_ABC"] + pre_t_A + pre["t_2"] for x in norm_cut_ABC]
    else:
        abs_cut_ABC = [float(x) for x in cut_ABC]
        norm_cut_ABC = [(float(x) - pre_t_A - pre["t_2"]) / pre["N_ABC"] for x in abs_cut_ABC]
        norm_cut_ABC.append(float("inf"))

    if "t_upper" not in optimized:  # the fixed-t_upper branch is unreachable (quirk 6)
        print("Warning: 't_upper' not found in parameter definition. Calculating from 't_3' "
              "and 'N_ABC'.")
        if "N_ABC" in optimized or "N_ABC" in fixed:
            n_abc = optimized["N_ABC"] if "N_ABC" in optimized else fixed["N_ABC"]
            t3 = optimized.get("t_3", fixed.get("t_3"))
            if t3 is None:
                raise ValueError("'t_3' not found in parameter definition.")
            optim_vars.append("t_upper")
            optim_vals.append(t3 - norm_cut_ABC[-2] * n_abc)
        else:
            raise ValueError("'N_ABC' not found in parameter definition.")
    else:
        optim_vars.append("t_upper")
        optim_vals.append(optimized["t_upper"])
    for i, p in enumerate(optim_vars):
        d[p] = optim_vals[i]
    if proportional_tm:
        if case == frozenset(["t_1"]):
            if d["t_m"] > 1:
                raise ValueError("If proportional t_m is wanted, please input t_m as a "
                                 "proportion (between 0 and 1).")
            d["t_m"] = d["t_1"] * d["t_m"]
        else:
            raise ValueError("Proportional t_m is only supported for the case where only "
                             "'t_1' is given, please input t_m as an absolute value (in "
                             "generations) if you also input 't_A', 't_B' or 't_C'.")
    for p in list(d):
        if p not in ("n_int_AB", "n_int_ABC"):
            d[p] = float(d[p]) / mu if p == "r" else float(d[p]) * mu
    if d["t_upper"] < 0:
        raise ValueError("Parameter 't_upper' must be a positive number. "
                         f"Given/calculated value: {d['t_upper']}")
    d = derive_times_int(d, case, norm_cut_ABC[-2])

    lo, hi = pre_t_A, pre_t_A + pre["t_2"]
    early = abs_cut_AB[0] < lo and not math.isclose(abs_cut_ABC[0], lo, rel_tol=1e-9, abs_tol=1e-12)
    late = abs_cut_AB[-1] > hi and not math.isclose(abs_cut_ABC[-1], hi, rel_tol=1e-9, abs_tol=1e-12)
    if early or late:
        raise ValueError("cutpoints_AB must lie within [t_A, t_A + t_2]."
                         f"Given cutpoints_AB: {abs_cut_AB}, t_A: {lo}, t_A + t_2: {hi}.")
    lo, hi = pre_t_A + pre["t_2"], d["t_out"] / mu
    early = abs_cut_ABC[0] < lo and not math.isclose(abs_cut_ABC[0], lo, rel_tol=1e-9, abs_tol=1e-12)
    late = abs_cut_ABC[-2] > hi and not math.isclose(abs_cut_ABC[-2], hi, rel_tol=1e-9, abs_tol=1e-12)
    if early or late:
        raise ValueError("cutpoints_ABC must lie within [t_A + t_2, t_out]."
                         f"Given cutpoints_ABC: {abs_cut_ABC}, t_A + t_2: {lo}, t_out: {hi}.")
    if verbose:
        print("Parameters validated:")
        print(f"Cutpoints AB: {abs_cut_AB}")
        print(f"Cutpoints ABC: {abs_cut_ABC}")
        for k, v in d.items():
            if k in ("n_int_AB", "n_int_ABC"):
                print(f"{k}: {v}")
            else:
                print(f"{k}: {v * mu if k == 'r' else v / mu}")
    d.pop("n_int_AB")
    d.pop("n_int_ABC")
    s.params = d
    s.norm_cut_AB, s.norm_cut_ABC = norm_cut_AB, norm_cut_ABC
    s.abs_cut_AB, s.abs_cut_ABC = abs_cut_AB, abs_cut_ABC
    return s


# ---------------------------------------------------------------------------------------
# optimizer CLI (itrails-optimize)
# ---------------------------------------------------------------------------------------
class OptimizeSetup:
    def __init__(self):
        self.maf_path = ""
        self.output = ""
        self.output_dir = ""
        self.output_prefix = ""
        self.species_list: List[str] = []
        self.method = "nelder-mead"
        self.optim_variables: List[str] = []
        self.optim_list: List[float] = []
        self.bounds: List[Tuple[float, float]] = []
        self.fixed: Dict = {}          # internal units + n_int_AB / n_int_ABC
        self.case = frozenset()
        self.mu = 0.0
        self.n_cpu = 1
        self.starting_params: Dict = {}
        self.best_model: Dict = {}


def resolve_optimize(config: Dict, input_cmd=None, output_cmd=None,
                     intro: bool = False) -> OptimizeSetup:
    """workflow_optimize.py:46-470 up to (not including) reading the MAF and minimising.
    intro=True: itrails-int-optimize (workflow_int_optimize.py:46-455) — t_m, N_BC and m
    are mandatory (m is mu-scaled like the others), settings.proportional is rejected, and
    the reference's t_upper negativity checks are absent."""
    s = OptimizeSetup()
    settings = config["settings"]
    s.maf_path, s.output = resolve_io(input_cmd, output_cmd, settings["input_maf"],
                                      settings["output_prefix"])
    s.output_dir, s.output_prefix = os.path.split(s.output)
    os.makedirs(s.output_dir, exist_ok=True)
    print(f"Results will be saved to: {s.output_dir}.")
    requested = settings.get("n_cpu")
    s.n_cpu = update_n_cpu(requested)
    if requested is None:
        print(f"No CPU count specified in config; using default {s.n_cpu} cores.")
    if intro and settings.get("proportional"):
        raise ValueError("Proportional t_m is currently not supported in the optimization "
                         "workflow. Please provide t_m as an absolute value in generations.")
    fixed, optimized = config["fixed_parameters"], config["optimized_parameters"]
    settings["output_prefix"] = s.output
    settings["input_maf"] = s.maf_path
    settings["n_cpu"] = s.n_cpu
    s.species_list = settings["species_list"]
    mu = float(fixed["mu"])
    s.mu = mu
    n_int_AB, n_int_ABC = settings["n_int_AB"], settings["n_int_ABC"]
    d: Dict = {}
    if not (isinstance(n_int_AB, int) and n_int_AB > 0):
        raise ValueError("n_int_AB must be a positive integer")
    d["n_int_AB"] = n_int_AB
    if not (isinstance(n_int_ABC, int) and n_int_ABC > 0):
        raise ValueError("n_int_ABC must be a positive integer")
    d["n_int_ABC"] = n_int_ABC
    if mu <= 0:
        raise ValueError("mu must be a positive float or int.")
    method = settings["method"].lower()
    allowed = ["nelder-mead", "l-bfgs-b"]
    if method not in allowed:
        raise ValueError(f"Method must be one of {allowed}.")
    print(f"Using optimization method: {method}")
    s.method = method

    found: set = set()
    tv = _time_values(fixed, optimized, found, with_bounds=True)
    if frozenset(found) not in TIME_COMBINATIONS:
        raise ValueError(f"Invalid combination of time values: {found}, check possible "
                         "combinations in the documentation.")
    names, start, bounds = [], [], []
    for p in ("t_1", "t_A", "t_B", "t_C"):
        if p in found:
            v, lo, hi, is_fixed = tv[p]
            if is_fixed:
                d[p] = v
            else:
                names.append(p)
                start.append(v)
                bounds.append((lo, hi))
    s.case = frozenset(found)
    for p in (INT_CORE_PARAMS if intro else CORE_PARAMS):
        if p in fixed and p in optimized:
            raise ValueError(f"Parameter '{p}' cannot be both fixed and optimized.")
        if p in fixed:
            d[p] = fixed[p]
        elif p in optimized:
            names.append(p)
            start.append(optimized[p][0])
            bounds.append((optimized[p][1], optimized[p][2]))
        elif intro:
            raise ValueError("Parameters 't_2', 'N_ABC', 'N_AB', 'N_BC', 't_m', 'm' and 'r' "
                             "must be present in optimized or fixed parameters.")
        else:
            raise ValueError("Parameters 't_2', 'N_ABC', 'N_AB' and 'r' must be present in "
                             "optimized or fixed parameters.")

    def last_cut(n_abc):  # cutpoints_ABC(n, 1 / N_ABC)[-2]
        return cutpoints_ABC(d["n_int_ABC"], 1 / n_abc)[-2]

    if "t_upper" not in optimized:
        print("Warning: 't_upper' not found in parameter definition. Calculating from 't_3' "
              "and 'N_ABC'.")
        if "N_ABC" in optimized:
            n0, n_lo, n_hi = optimized["N_ABC"]
            if "t_3" in optimized:
                t3, t3_lo, t3_hi = optimized["t_3"]
            elif "t_3" in fixed:
                t3 = t3_lo = t3_hi = fixed["t_3"]
            else:
                raise ValueError("'t_3' not found in parameter definition.")
            tu = [t3 - last_cut(n0), t3_lo - last_cut(n_hi), t3_hi - last_cut(n_lo)]
        elif "N_ABC" in fixed:
            n0 = fixed["N_ABC"]
            if "t_3" in optimized:
                t3, t3_lo, t3_hi = optimized["t_3"]
                tu = [t3 - last_cut(n0), t3_lo - last_cut(n0), t3_hi - last_cut(n0)]
            elif "t_3" in fixed:
                raise ValueError("At least one, 't_3' or 'N_ABC' must be present in optimized "
                                 "parameters.")
            else:
                raise ValueError("'t_3' not found in parameter definition.")
        else:
            raise ValueError("'N_ABC' not found in parameter definition.")
        if not (tu[1] <= tu[0] <= tu[2]):
            raise ValueError(f"When calculating t_upper from t_3 and N_ABC, the starting value "
                             f"({tu[0]}) was not between the minimum ({tu[1]}) and maximum "
                             f"({tu[2]}).")
        if min(tu) < 0 and not intro:
            raise ValueError("Calculated 't_upper' values cannot be negative. Please check your "
                             "input parameters.")
        names.append("t_upper")
        # workflow_optimize.py:311: with N_ABC fixed and t_3 optimized the reference appends
        # the whole [start, lo, hi] list as the start value; that path then fails in its
        # float() check below exactly as here
        start.append(tu if ("N_ABC" in fixed and "t_3" in optimized) else tu[0])
        bounds.append((tu[1], tu[2]))
    else:
        v = optimized["t_upper"]
        names.append("t_upper")
        start.append(v[0])
        bounds.append((v[1], v[2]))
        if (v[0] < 0 or v[1] < 0 or v[2] < 0) and not intro:
            raise ValueError("Parameter 't_upper' cannot be negative. Please check your input "
                             "parameters.")
    if "t_out" in fixed:
        d["t_out"] = fixed["t_out"]
    elif "t_out" in optimized:
        raise ValueError("Parameter 't_out' has to be fixed.")

    for i, p in enumerate(names):
        if p in fixed:
            raise ValueError(f"Parameter '{p}' cannot be present in both fixed and optimized "
                             "parameters.")
        v, lo, hi = float(start[i]), float(bounds[i][0]), float(bounds[i][1])
        if not (lo <= v <= hi):
            raise ValueError(f"Starting value for '{p}' ({v}) must be between the minimum "
                             f"({lo}) and maximum ({hi}).")
        if v <= 0:
            raise ValueError(f"Starting value for '{p}' must be a positive number.")
        if lo <= 0:
            raise ValueError(f"Minimum value for '{p}' must be a positive number.")
        f = (1 / mu) if p == "r" else mu
        start[i], bounds[i] = v * f, (lo * f, hi * f)
    for p in list(d):
        if p not in ("n_int_AB", "n_int_ABC"):
            d[p] = float(d[p]) / mu if p == "r" else float(d[p]) * mu

    user_fixed = {k: (v * mu if k == "r" else v / mu) for k, v in d.items()
                  if k not in ("n_int_AB", "n_int_ABC")}
    user_fixed["mu"] = mu
    back = lambda v, p: float(v) * mu if p == "r" else float(v) / mu  # noqa: E731
    starting = {p: FlowSeq([back(start[i], p), back(bounds[i][0], p), back(bounds[i][1], p)])
                for i, p in enumerate(names)}
    if "species_list" in settings:
        settings["species_list"] = FlowSeq(settings["species_list"])
    s.starting_params = {"fixed_parameters": user_fixed, "optimized_parameters": starting,
                         "settings": settings}
    s.best_model = {"fixed_parameters": user_fixed, "optimized_parameters": {},
                    "results": {"log_likelihood": -math.inf, "iteration": None},
                    "settings": settings}
    s.optim_variables, s.optim_list, s.bounds, s.fixed = names, start, bounds, d
    return s
