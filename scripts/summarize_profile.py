"""Condense a rocprofv3 output directory (kernel-trace stats + FETCH_SIZE / WRITE_SIZE PMC
passes written by scripts/gpu_profile.sh) into profiles/<tag>_*.{csv,json}.

FETCH_SIZE / WRITE_SIZE are in KiB per dispatch.  The gfx950 x2 correction for FETCH_SIZE
(MI355X_MICROARCH.md, HBM section) is calibrated for 16-B-per-lane streaming reads; the
sweep kernels' HBM reads are 2-B-per-lane symbol loads, for which the raw FETCH_SIZE already
matches the symbol array size (10 M columns x 2 B = 20.0 MB vs 21.6 MB measured), so the raw
value is reported and the corrected one is listed beside it.
"""
import csv
import collections
import json
import os
import shutil
import sys


def main(prof_dir, tag, n_states=None, out_dir="profiles"):
    os.makedirs(out_dir, exist_ok=True)
    stats = os.path.join(prof_dir, "trace_kernel_stats.csv")
    shutil.copy(stats, os.path.join(out_dir, f"{tag}_kernel_stats.csv"))
    per = collections.defaultdict(dict)
    for r in csv.DictReader(open(stats)):
        per[r["Name"]].update(calls=int(r["Calls"]), avg_ns=float(r["AverageNs"]))
    for fname, key in (("pmc_fetch_counter_collection.csv", "FETCH_SIZE"),
                       ("pmc_write_counter_collection.csv", "WRITE_SIZE")):
        vals = collections.defaultdict(list)
        for r in csv.DictReader(open(os.path.join(prof_dir, fname))):
            if r["Counter_Name"] == key:
                vals[r["Kernel_Name"]].append(float(r["Counter_Value"]))
        for k, v in vals.items():
            per[k][key + "_KiB"] = sum(v) / len(v)
    for k, d in per.items():
        if "FETCH_SIZE_KiB" in d and "WRITE_SIZE_KiB" in d:
            d["hbm_bytes_raw"] = 1024 * (d["FETCH_SIZE_KiB"] + d["WRITE_SIZE_KiB"])
            d["hbm_bytes_fetch_x2"] = 1024 * (2 * d["FETCH_SIZE_KiB"] + d["WRITE_SIZE_KiB"])
    if n_states is not None:  # model size of the profiled command (bench.py pmc_traffic)
        for d in per.values():
            d["n_states"] = n_states
    json.dump(per, open(os.path.join(out_dir, f"{tag}_summary.json"), "w"), indent=1)
    print(json.dumps(per, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], int(sys.argv[3]) if len(sys.argv) > 3 else None)
