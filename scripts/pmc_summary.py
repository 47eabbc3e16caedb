"""Condense rocprofv3 --pmc passes (one counter_collection.csv per pass, any number of passes
over the same command) and the --kernel-trace --stats summary into one JSON per kernel:
per-dispatch averages of every counter plus derived rates.

usage: python scripts/pmc_summary.py <prof_dir> <out.json> [kernel-substring ...]

Units (MI355X_MICROARCH.md, rocprofv3 PMC): SQ_WAVE_CYCLES / SQ_BUSY_CYCLES / SQ_WAIT_* /
SQ_ACTIVE_INST_* count quad-cycles (x4 = shader cycles); SQ_VALU_MFMA_BUSY_CYCLES counts
cycles; GRBM_GUI_ACTIVE is summed over the 8 XCDs (/8 = the dispatch's wall cycles).
Derived (per dispatch):
  valu_issue_util  SQ_ACTIVE_INST_VALU x4 / (wall cycles x SIMDs): share of SIMD-cycles
                   that issued a VALU instruction (wave-level; an FP64 wave-instruction
                   occupies the SIMD ~4 cycles, so x4 of the issue count is the FP64 busy share)
  valu_busy        SQ_INSTS_VALU x 4 cycles / (wall cycles x SIMDs): FP64 VALU occupancy if
                   every VALU instruction is a 4-cycle FP64 one (upper bound for mixed code)
  mfma_util        SQ_VALU_MFMA_BUSY_CYCLES / (wall cycles x SIMDs)
  wait_share       SQ_WAIT_ANY / SQ_WAVE_CYCLES (waves parked on s_waitcnt / barrier)
  inst_stall_share SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES (issue stalls: dependency / pipe busy)
"""
import collections
import csv
import glob
import json
import os
import sys

SIMDS = 256 * 4


def main(prof_dir, out, subs):
    per = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(os.path.join(prof_dir, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"]
            if subs and not any(s in k for s in subs):
                continue
            per[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    stats = {}
    for f in glob.glob(os.path.join(prof_dir, "**", "*kernel_stats.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            stats[r["Name"]] = dict(calls=int(r["Calls"]), avg_ns=float(r["AverageNs"]))
    res = {}
    for k, d in per.items():
        avg = {c: sum(v) / len(v) for c, v in d.items()}
        e = {"counters": {c: round(v, 1) for c, v in sorted(avg.items())},
             "dispatches": max(len(v) for v in d.values())}
        if k in stats:
            e.update(stats[k])
        wall = avg.get("GRBM_GUI_ACTIVE", 0.0) / 8.0
        if wall > 0:
            e["wall_cycles"] = round(wall)
            if "SQ_ACTIVE_INST_VALU" in avg:
                e["valu_issue_util"] = round(avg["SQ_ACTIVE_INST_VALU"] * 4 / (wall * SIMDS), 4)
            if "SQ_INSTS_VALU" in avg:
                e["valu_busy"] = round(avg["SQ_INSTS_VALU"] * 4 / (wall * SIMDS), 4)
            if "SQ_VALU_MFMA_BUSY_CYCLES" in avg:
                e["mfma_util"] = round(avg["SQ_VALU_MFMA_BUSY_CYCLES"] / (wall * SIMDS), 4)
        if avg.get("SQ_WAVE_CYCLES"):
            for c, name in (("SQ_WAIT_ANY", "wait_share"), ("SQ_WAIT_INST_ANY", "inst_stall_share"),
                            ("SQ_ACTIVE_INST_ANY", "active_share")):
                if c in avg:
                    e[name] = round(avg[c] / avg["SQ_WAVE_CYCLES"], 4)
        # HBM bytes (KiB counters; FETCH_SIZE x2 is the gfx950 correction for 16-B-per-lane
        # streaming reads, MI355X_MICROARCH.md — the sweeps' reads are mostly narrower, so
        # both are kept)
        if "FETCH_SIZE" in avg and "WRITE_SIZE" in avg:
            e["FETCH_SIZE_KiB"] = round(avg["FETCH_SIZE"], 1)
            e["WRITE_SIZE_KiB"] = round(avg["WRITE_SIZE"], 1)
            e["hbm_bytes_raw"] = round(1024 * (avg["FETCH_SIZE"] + avg["WRITE_SIZE"]))
            e["hbm_bytes_fetch_x2"] = round(1024 * (2 * avg["FETCH_SIZE"] + avg["WRITE_SIZE"]))
        # state count of the profiled launch: the (7,7) model's kernels carry NT = 9 tiles
        e["n_states"] = 133 if ("<9, 34," in k or "<9, 36," in k) else 70
        res[k] = e
    for k, e in res.items():
        print(k[:100])
        print("   ", {x: y for x, y in e.items() if x != "counters"})
    # the library the profiled command loaded (bench.py prefers the summary of its own build)
    lib = os.environ.get("ITR_LIB") or os.path.join(os.path.dirname(os.path.abspath(__file__)),
                                                     "..", "itrails_amd", "libitrails_hip.so")
    if os.path.exists(lib):
        import hashlib
        res["library_sha256"] = hashlib.sha256(open(lib, "rb").read()).hexdigest()
    json.dump(res, open(out, "w"), indent=1)


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], sys.argv[3:])
