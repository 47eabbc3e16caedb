"""HBM bytes per itr_forward_viterbi call from the FETCH_SIZE / WRITE_SIZE passes of the
default bench command (scripts/r4/final.sh: rocprofv3 --pmc FETCH_SIZE, then WRITE_SIZE,
over `bench.py --steps 3 --warmup 1 --verify 0`): every launch of the call's kernels — the
mixed launch and the two reserved sets' late launches (wave_mixed_kernel, roles 0/1/2), the
long blocks' Viterbi sweep (vit_group_kernel; sweep_kernel<VIT> before round 6) and the
forward's VALU halves (fwd_group_kernel; hybrid_sweep_kernel<FWD_LL> before) — divided by the number of calls (one role-0 mixed launch per
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


def lib_sha256(path=None):
    import hashlib
    path = path or os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "itrails_amd", "libitrails_hip.so")
    return hashlib.sha256(open(path, "rb").read()).hexdigest()


def main(prof, out):
    tot = {"FETCH_SIZE": collections.defaultdict(float), "WRITE_SIZE": collections.defaultdict(float)}
    disp = collections.Counter()
    for f in glob.glob(os.path.join(prof, "*counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"]
            tot[r["Counter_Name"]][k] += float(r["Counter_Value"])
            if r["Counter_Name"] == "FETCH_SIZE":
                disp[k] += 1
    calls = sum(n for k, n in disp.items() if "wave_mixed_kernel" in k and ", 0>(" in k)
    parts = {}
    for c, d in tot.items():
        for k, v in d.items():
            if "wave_mixed_kernel" in k:
                per = v * 1024 / calls
            elif ("sweep_kernel<" in k and k.endswith(", 3>(itr::SweepArgs)")) or \
                    ("hybrid_sweep_kernel<" in k and ", 0, 2," in k) or \
                    "vit_group_kernel<" in k or "fwd_group_kernel<" in k:
                per = v * 1024 / disp[k]
            else:
                continue
            parts.setdefault(k, {})[c] = per
    fetch = sum(p.get("FETCH_SIZE", 0.0) for p in parts.values())
    write = sum(p.get("WRITE_SIZE", 0.0) for p in parts.values())
    res = {"calls": calls, "bytes_per_call": round(2 * fetch + write),
           "fetch_raw": round(fetch), "write_raw": round(write),
           "per_kernel": {k: {c: round(v) for c, v in p.items()} for k, p in parts.items()},
           "library_sha256": lib_sha256(),
           "source": os.path.relpath(prof),
           "units": "bytes per call: 2 x FETCH_SIZE + WRITE_SIZE (KiB x 1024; gfx950 FETCH "
                    "correction, MI355X_MICROARCH.md HBM section)"}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
