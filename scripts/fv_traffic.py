"""HBM bytes per itr_forward_viterbi call from the FETCH_SIZE / WRITE_SIZE passes of the
default bench command (scripts/r4/final.sh: rocprofv3 --pmc FETCH_SIZE, then WRITE_SIZE,
over `bench.py --steps 3 --warmup 1 --verify 0`): every launch of the call's kernels — the
mixed launch and the two reserved sets' late launches (wave_mixed_kernel, roles 0/1/2), the
long blocks' Viterbi sweep (sweep_kernel<VIT>) and the forward's VALU halves
(hybrid_sweep_kernel<FWD_LL>) — divided by the number of calls (one role-0 mixed launch per
call).  The two non-mixed kernels also run in the bench's separate forward / Viterbi timing
calls, so they are counted at their per-dispatch average, once per call.  Units: the
counters report KiB (MI355X_MICROARCH.md); raw, no gfx950 FETCH correction applied.

usage: python scripts/fv_traffic.py <prof_dir> <out.json>"""
import collections
import csv
import glob
import json
import os
import sys


def main(prof, out):
    tot = collections.defaultdict(float)
    disp = collections.Counter()
    for f in glob.glob(os.path.join(prof, "*counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"]
            tot[k] += float(r["Counter_Value"])
            if r["Counter_Name"] == "FETCH_SIZE":
                disp[k] += 1
    calls = sum(n for k, n in disp.items() if "wave_mixed_kernel" in k and ", 0>(" in k)
    parts = {}
    for k, v in tot.items():
        if "wave_mixed_kernel" in k:
            parts[k] = v * 1024 / calls
        elif ("sweep_kernel<" in k and k.endswith(", 3>(itr::SweepArgs)")) or \
                ("hybrid_sweep_kernel<" in k and ", 0, 2," in k):
            parts[k] = v * 1024 / disp[k]
    res = {"calls": calls, "bytes_per_call": round(sum(parts.values())),
           "per_kernel": {k: round(v) for k, v in parts.items()},
           "source": os.path.relpath(prof), "units": "FETCH_SIZE + WRITE_SIZE (KiB x 1024), raw"}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
