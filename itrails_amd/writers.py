"""Result files of itrails-viterbi / itrails-posterior through the native writers
(itrails_amd/csrc/writers.cpp): byte-identical to the reference's csv.writer output
(workflow_viterbi.py:636-743, workflow_posterior.py:636-716)."""
from __future__ import annotations

import csv
import ctypes
from typing import Optional, Sequence

import numpy as np

from ._lib import check, lib

TOPOLOGY = {0: "({sp1,sp2},sp3)", 1: "((sp1,sp2),sp3)", 2: "((sp1,sp3),sp2)",
            3: "((sp2,sp3),sp1)"}
# the introgression CLIs add the introgressed V0 topology (workflow_int_viterbi.py:666-673)
TOPOLOGY_INT = {**TOPOLOGY, 4: "({sp2,sp3},sp1)"}


def _flat(blocks, dtype):
    off = np.zeros(len(blocks) + 1, dtype=np.int64)
    np.cumsum([len(b) for b in blocks], out=off[1:])
    flat = np.concatenate([np.asarray(b) for b in blocks]).astype(dtype) if off[-1] else \
        np.zeros(0, dtype=dtype)
    return flat, off


def format_float(x: float) -> str:
    """Python repr(float) as the native writer prints it."""
    buf = ctypes.create_string_buffer(40)
    check(lib().itr_format_float(float(x), buf, 40))
    return buf.value.decode()


def write_viterbi_csv(output_file: str, viterbi_result, ref_coordinates=None,
                      block_off: Optional[np.ndarray] = None):
    """viterbi_result: list of per-block state arrays (as viterbi_wrapper returns), or a
    flat uint8 path with `block_off`; ref_coordinates: parse_coordinates output (list of
    per-block lists) or a flat int64 array aligned with the columns."""
    if block_off is None:
        states, off = _flat(viterbi_result, np.uint8)
    else:
        states, off = np.ascontiguousarray(viterbi_result, dtype=np.uint8), np.asarray(block_off, np.int64)
    coords = None
    if ref_coordinates is not None:
        coords = ref_coordinates if isinstance(ref_coordinates, np.ndarray) else \
            _flat(ref_coordinates, np.int64)[0]
        coords = np.ascontiguousarray(coords, dtype=np.int64)
        if len(coords) != len(states):
            raise ValueError("reference coordinates do not match the decoded columns")
    check(lib().itr_write_viterbi_csv(str(output_file).encode(), states.ctypes.data,
                                      off.ctypes.data, len(off) - 1,
                                      coords.ctypes.data if coords is not None else None,
                                      len(coords) if coords is not None else 0))


def write_posterior_csv(output_file: str, posterior_results, ref_coordinates=None,
                        block_off: Optional[np.ndarray] = None, threads: int = 16):
    """posterior_results: list of T x N arrays (post_prob_wrapper) or a flat (columns x N)
    array with `block_off`."""
    if block_off is None:
        n = posterior_results[0].shape[1] if len(posterior_results) else 0
        post, off = _flat([np.asarray(p).reshape(-1, n) if n else np.zeros((len(p), 0))
                           for p in posterior_results], np.float64)
    else:
        post, off = np.asarray(posterior_results, np.float64), np.asarray(block_off, np.int64)
        n = post.shape[1] if post.ndim == 2 else 0
    post = np.ascontiguousarray(post, dtype=np.float64)
    coords = None
    if ref_coordinates is not None:
        coords = ref_coordinates if isinstance(ref_coordinates, np.ndarray) else \
            _flat(ref_coordinates, np.int64)[0]
        coords = np.ascontiguousarray(coords, dtype=np.int64)
        if len(coords) != len(post):
            raise ValueError("reference coordinates do not match the decoded columns")
    if len(post) != (int(off[-1]) if len(off) else 0):
        raise ValueError("posterior rows do not match the block offsets")
    check(lib().itr_write_posterior_csv(str(output_file).encode(), post.ctypes.data, int(n),
                                        off.ctypes.data, len(off) - 1,
                                        coords.ctypes.data if coords is not None else None,
                                        len(coords) if coords is not None else 0,
                                        int(threads)))


def write_hidden_states_csv(output_file: str, hidden_names: dict, abs_cut_AB: Sequence[float],
                            abs_cut_ABC: Sequence[float], posterior: bool):
    """hidden_states.csv (workflow_viterbi.py:636-684 / workflow_posterior.py:636-685);
    V0 first-coalescent intervals use the ABC cutpoints for Viterbi and the AB cutpoints for
    posterior decoding."""
    with open(output_file, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["state_idx", "topology", "interval_1st_coalescent",
                    "interval_2nd_coalescent", "shorthand_name"])
        for idx, sh in hidden_names.items():
            k = sh[0]
            cut1 = abs_cut_AB if (posterior and k == 0) else abs_cut_ABC
            t1 = f"{cut1[sh[1]]:.2f}-{cut1[sh[1] + 1]:.2f}"
            t2 = f"{abs_cut_ABC[sh[2]]:.2f}-{abs_cut_ABC[sh[2] + 1]:.2f}"
            w.writerow([idx, TOPOLOGY.get(k, "Unknown"), t1, t2, sh])


def write_hidden_states_csv_int(output_file: str, hidden_names: dict,
                                abs_cut_AB: Sequence[float], abs_cut_ABC: Sequence[float]):
    """hidden_states.csv of itrails-int-viterbi / itrails-int-posterior
    (workflow_int_viterbi.py:666-712): written through pandas there, so '\\n' line ends;
    the first-coalescent interval uses the AB cutpoints for topology 0 and the ABC
    cutpoints for every other topology — the introgressed states (4, i, j) included,
    although their i indexes a BC interval (kept as the reference labels it)."""
    with open(output_file, "w", newline="") as f:
        w = csv.writer(f, lineterminator="\n")
        w.writerow(["state_idx", "topology", "interval_1st_coalescent",
                    "interval_2nd_coalescent", "shorthand_name"])
        for idx, sh in hidden_names.items():
            k, i1, i2 = sh
            cut1 = abs_cut_AB if k == 0 else abs_cut_ABC
            t1 = f"{cut1[i1]:.2f}-{cut1[i1 + 1]:.2f}"
            t2 = f"{abs_cut_ABC[i2]:.2f}-{abs_cut_ABC[i2 + 1]:.2f}"
            w.writerow([idx, TOPOLOGY_INT.get(k, "Unknown"), t1, t2, sh])
