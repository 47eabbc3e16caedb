"""BASELINE config 1 end to end through the drop-in CLI: a synthetic (5,5) MAF (default 100
kbp, sampled from the reference's (5,5) KAT model with gaps and Ns) decoded by
`python -m itrails_amd viterbi` (= itrails-viterbi: YAML resolution, device model build,
MAF ingest, Viterbi sweep + traceback, hidden_states.csv + viterbi.csv), wall time of the
whole command measured around the child process.  The reference's own path for the same
command is dominated by its (5,5) model build (615 s on the 8-core build container,
BASELINE.md 2), cited, not re-run here (it cannot run on the GPU box).

usage: python scripts/cli_e2e.py [kbp] [out.json]"""
import json
import os
import subprocess
import sys
import tempfile
import time

import numpy as np
import yaml

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from itrails_amd.synth import block_lengths, sample_alignment, write_maf  # noqa: E402

SP = ["hg38", "panTro5", "gorGor5", "ponAbe2"]


def main():
    kbp = float(sys.argv[1]) if len(sys.argv) > 1 else 100.0
    out = sys.argv[2] if len(sys.argv) > 2 else None
    g = np.load(os.path.join(ROOT, "tests", "golden", "model_kat_5_5.npz"))
    tmp = tempfile.mkdtemp()
    lengths = block_lengths(np.random.default_rng(21), int(kbp * 1000), 2000.0)
    obs, off, _ = sample_alignment(g["a"], g["b"], g["pi"], lengths, seed=22)
    maf = os.path.join(tmp, "chr.maf")
    write_maf(maf, obs, off, SP, seed=23)
    cfg = {"fixed_parameters": {"mu": 2e-8, "t_1": 240000.0, "t_2": 40000.0, "N_AB": 50000.0,
                                "N_ABC": 50000.0, "r": 1e-8},
           "optimized_parameters": {"t_upper": 745069.3855},
           "settings": {"input_maf": maf, "output_prefix": os.path.join(tmp, "out", "run"),
                        "species_list": SP, "n_int_AB": 5, "n_int_ABC": 5, "n_cpu": 16,
                        "reference": "hg38"}}
    cf = os.path.join(tmp, "cfg.yaml")
    yaml.dump(cfg, open(cf, "w"))
    cmd = [sys.executable, "-m", "itrails_amd", "viterbi", "--config-file", cf]
    runs = []
    for _ in range(2):  # the first run also pays the process start and first-use costs
        t0 = time.perf_counter()
        subprocess.run(cmd, check=True, cwd=ROOT, stdout=subprocess.DEVNULL)
        runs.append(time.perf_counter() - t0)
    res = {"workload": f"itrails-viterbi, (5,5) model, {kbp:g} kbp synthetic MAF "
                       f"({len(lengths)} blocks), reference coordinates",
           "wall_seconds_per_run": [round(r, 3) for r in runs],
           "columns": int(off[-1]),
           "reference_model_build_seconds": 615.0,
           "note": "whole command incl. python start, YAML, device model build, MAF read, "
                   "decode, CSV writes; reference: (5,5) trans_emiss_calc alone 615 s on 8 "
                   "cores (BASELINE.md 2)"}
    print(json.dumps(res))
    if out:
        json.dump(res, open(out, "w"), indent=1)


if __name__ == "__main__":
    main()
