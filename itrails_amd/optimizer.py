"""The maximum-likelihood loop of itrails-optimize (optimizer.py:380-637) on the device path.

Each objective evaluation rebuilds the HMM with the device model build
(itrails_amd.model.trans_emiss_calc: batched Pade expm / Van Loan / emission kernels) and
evaluates the forward log-likelihood of every block with the sweep kernel on columns that
stay resident in HBM for the whole run; the host keeps the reference's bookkeeping
(optimization_history.csv rows, best_model.yaml updates, scipy.optimize.minimize).
Multi-GPU: with torch.distributed initialised, every rank holds a column-balanced shard of
the blocks and the per-block log-likelihoods are exchanged with one all-reduce
(itrails_amd.distributed), so every rank sees the same objective value.
"""
from __future__ import annotations

import os
import time
from typing import Dict, List, Optional, Sequence

import numpy as np

from . import hmm
from .config import derive_times, derive_times_int, update_best_model
from .model.emissions import cutpoints_ABC
from .model.trans_emiss import trans_emiss_calc


def write_list(lst: Sequence, res_name: str) -> None:
    """optimizer.py:380-393: append one comma-separated line (str() of each value)."""
    with open(res_name, "a") as f:
        f.write(",".join(str(v) for v in lst) + "\n")


class DeviceAlignment:
    """The blocks of one alignment resident on the current device (or this rank's shard
    of them): symbols (uint16) and a plan, reused by every objective evaluation."""

    def __init__(self, V_lst: Sequence[np.ndarray], group=None):
        import torch
        import torch.distributed as dist

        self.nblocks_total = len(V_lst)
        self.lo, self.hi = 0, len(V_lst)
        self.dist = dist.is_available() and dist.is_initialized()
        self.group = group
        if self.dist:
            from .distributed import shard_ranges

            ranges = shard_ranges([len(v) for v in V_lst], dist.get_world_size(group))
            self.lo, self.hi = ranges[dist.get_rank(group)]
        obs, off = hmm.concat_blocks(list(V_lst[self.lo:self.hi]))
        self.plan = hmm.Plan(off)
        dev = torch.device("cuda", torch.cuda.current_device())
        self.d_obs = torch.from_numpy(obs.astype(np.int16)).to(dev)
        self.d_ll = torch.empty(max(self.plan.nblocks, 1), dtype=torch.float64, device=dev)

    def block_logliks(self, a, b, pi) -> np.ndarray:
        """Per-block log-likelihoods of ALL blocks (every rank gets the full vector)."""
        import torch

        model = hmm.Model(a, b, pi)
        try:
            if self.plan.nblocks:
                hmm.forward_loglik_device(model, self.plan, self.d_obs, out=self.d_ll)
            local = self.d_ll[: self.plan.nblocks].cpu().numpy()
        finally:
            model.close()
        if not self.dist:
            return local
        from .distributed import _comm_device, gather_block_values

        return gather_block_values(local, self.lo, self.nblocks_total, group=self.group,
                                   device=_comm_device())

    def loglik(self, a, b, pi) -> float:
        """loglik_wrapper semantics: Python float, `acc +=` in block order."""
        acc = 0
        for v in self.block_logliks(a, b, pi).tolist():
            acc += v
        return acc


def model_for(arg_lst, optimized_params: Sequence[str], case: frozenset, d: Dict):
    """optimizer.py:419-555: the parameter dictionary of one evaluation and its HMM."""
    dd = dict(d)
    for i, p in enumerate(optimized_params):
        dd[p] = arg_lst[i]
    last = cutpoints_ABC(dd["n_int_ABC"], 1)[dd["n_int_ABC"] - 1]
    dd = derive_times(dd, case, last)
    return dd, trans_emiss_calc(dd["t_A"], dd["t_B"], dd["t_C"], dd["t_2"], dd["t_upper"],
                                dd["t_out"], dd["N_AB"], dd["N_ABC"], dd["r"],
                                dd["n_int_AB"], dd["n_int_ABC"], "standard", "standard")


def _nccl() -> bool:
    import torch.distributed as dist
    return dist.is_initialized() and dist.get_backend() == "nccl"


def optimization_wrapper(arg_lst, optimized_params, case, d, data: DeviceAlignment,
                         res_name: str, info: Dict) -> float:
    """optimizer.py:396-585: one objective evaluation -> -loglik, with the history row and
    the best-model update the reference writes (rank 0 only when distributed)."""
    output_dir, output_prefix = os.path.split(res_name)
    from .model.linalg import split_build
    # multi-GPU: the rebuild's Van Loan work is divided over the ranks (every rank
    # evaluates the same parameters at the same time)
    with split_build(data.dist and _nccl(), data.group):
        _, (a, b, pi, _, _) = model_for(arg_lst, optimized_params, case, d)
    loglik = data.loglik(a, b, pi)
    if _is_writer():
        write_list([info["Nfeval"]] + list(np.asarray(arg_lst).tolist()) +
                   [loglik, time.time() - info["time"]],
                   os.path.join(output_dir, f"{output_prefix}.optimization_history.csv"))
        update_best_model(os.path.join(output_dir, f"{output_prefix}.best_model.yaml"),
                          optimized_params, arg_lst, loglik, info["Nfeval"])
    info["Nfeval"] += 1
    return -loglik


def _is_writer() -> bool:
    try:
        import torch.distributed as dist

        return not (dist.is_available() and dist.is_initialized()) or dist.get_rank() == 0
    except Exception:
        return True


def optimizer(optim_variables: List[str], optim_list: List[float], bounds, fixed_params: Dict,
              V_lst, res_name: str, case: frozenset, method: str = "Nelder-Mead",
              header: bool = True, options: Optional[Dict] = None):
    """optimizer.py:588-637: minimise -loglik with scipy (maxiter 10000, disp) starting at
    optim_list; V_lst is the reference's list of symbol arrays (or a DeviceAlignment)."""
    from scipy.optimize import minimize

    output_dir, output_prefix = os.path.split(res_name)
    if header and _is_writer():
        write_list(["n_eval"] + list(optim_variables) + ["loglik", "time"],
                   os.path.join(output_dir, f"{output_prefix}.optimization_history.csv"))
    data = V_lst if isinstance(V_lst, DeviceAlignment) else DeviceAlignment(V_lst)
    opts = {"maxiter": 10000, "disp": True} if options is None else options
    return minimize(optimization_wrapper, x0=optim_list,
                    args=(optim_variables, case, dict(fixed_params), data, res_name,
                          {"Nfeval": 0, "time": time.time()}),
                    method=method, bounds=bounds, options=opts)


# ---------------------------------------------------------------------------------------
# introgression model (int_optimizer.py:397-651)
# ---------------------------------------------------------------------------------------


def model_for_introgression(arg_lst, optimized_params: Sequence[str], case: frozenset, d: Dict,
                            tmp_path: str = "./"):
    """int_optimizer.py:404-548: the parameter dictionary of one evaluation and its HMM."""
    from .model.intro import trans_emiss_calc_introgression

    dd = dict(d)
    for i, p in enumerate(optimized_params):
        dd[p] = arg_lst[i]
    last = cutpoints_ABC(dd["n_int_ABC"], 1)[dd["n_int_ABC"] - 1]
    dd = derive_times_int(dd, case, last)
    return dd, trans_emiss_calc_introgression(
        dd["t_A"], dd["t_B"], dd["t_C"], dd["t_2"], dd["t_upper"], dd["t_out"], dd["t_m"],
        dd["N_AB"], dd["N_BC"], dd["N_ABC"], dd["r"], dd["m"], dd["n_int_AB"],
        dd["n_int_ABC"], "standard", "standard", tmp_path)


def _write_state_tables(hidden_names: Dict, observed_names: Dict) -> None:
    """int_optimizer.py:549-559: the first evaluation writes hidden_states.csv and
    observed_states.csv into the working directory (pandas to_csv layout)."""
    import csv

    for name, col, table in (("hidden_states.csv", "hidden", hidden_names),
                             ("observed_states.csv", "observed", observed_names)):
        with open(name, "w", newline="") as f:
            w = csv.writer(f, lineterminator="\n")
            w.writerow(["idx", col])
            for k, v in table.items():
                w.writerow([k, v])


def optimization_wrapper_introgression(arg_lst, optimized_params, case, d,
                                       data: DeviceAlignment, res_name: str,
                                       info: Dict) -> float:
    """int_optimizer.py:397-586: one objective evaluation -> -loglik; history rows and the
    best model go to {prefix}_optimization_history.csv / {prefix}_best_model.yaml."""
    output_dir, output_prefix = os.path.split(res_name)
    _, (a, b, pi, hidden, observed) = model_for_introgression(
        arg_lst, optimized_params, case, d, info.get("tmp_path", "./"))
    if info["Nfeval"] == 0 and _is_writer():
        _write_state_tables(hidden, observed)
    loglik = data.loglik(a, b, pi)
    if _is_writer():
        write_list([info["Nfeval"]] + list(np.asarray(arg_lst).tolist()) +
                   [loglik, time.time() - info["time"]],
                   os.path.join(output_dir, f"{output_prefix}_optimization_history.csv"))
        update_best_model(os.path.join(output_dir, f"{output_prefix}_best_model.yaml"),
                          optimized_params, arg_lst, loglik, info["Nfeval"])
    info["Nfeval"] += 1
    return -loglik


def optimizer_introgression(optim_variables: List[str], optim_list: List[float], bounds,
                            fixed_params: Dict, V_lst, res_name: str, case: frozenset,
                            method: str = "Nelder-Mead", header: bool = True,
                            tmp_path: str = "./", options: Optional[Dict] = None):
    """int_optimizer.py:589-651 on the device path."""
    from scipy.optimize import minimize

    output_dir, output_prefix = os.path.split(res_name)
    if header and _is_writer():
        write_list(["n_eval"] + list(optim_variables) + ["loglik", "time"],
                   os.path.join(output_dir, f"{output_prefix}_optimization_history.csv"))
    data = V_lst if isinstance(V_lst, DeviceAlignment) else DeviceAlignment(V_lst)
    opts = {"maxiter": 10000, "disp": True} if options is None else options
    return minimize(optimization_wrapper_introgression, x0=optim_list,
                    args=(optim_variables, case, dict(fixed_params), data, res_name,
                          {"Nfeval": 0, "time": time.time(), "tmp_path": tmp_path}),
                    method=method, bounds=bounds, options=opts)
