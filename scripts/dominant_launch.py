"""The dominant launch of the default bench command's kernel trace, per phase: the bench runs
`warmup` untimed steps, `steps` timed steps, then 3 instrumented steps (separate forward and
Viterbi calls before the combined one), so the dominant kernel's dispatches split
[warmup | timed | instrumented].  Writes the per-phase means beside the bench line's numbers.
usage: python scripts/dominant_launch.py <kernel_trace.csv> <bench line json> <out json> [warmup steps]"""
import csv
import hashlib
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    trace, line, out = sys.argv[1:4]
    warm = int(sys.argv[4]) if len(sys.argv) > 4 else 10
    steps = int(sys.argv[5]) if len(sys.argv) > 5 else 20
    rows = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"])
            for r in csv.DictReader(open(trace))]
    tot = {}
    for s, e, n in rows:
        tot[n] = tot.get(n, 0) + e - s
    kern = max(tot, key=tot.get)
    d = [(e - s) / 1e6 for s, e, n in sorted(rows) if n == kern]
    timed = d[warm:warm + steps]
    b = json.loads([x for x in open(line) if x.startswith("{")][-1])
    r = b["roofline"]
    ideal = r.get("step_ideal_ms")
    lib = os.path.join(ROOT, "itrails_amd", "libitrails_hip.so")
    res = {
        "command": "rocprofv3 --kernel-trace --stats -- python3 bench.py --verify 0 "
                   "--cpu-1core-cols 0 --host-path 0 (the default 10 warmup + 20 timed steps, "
                   "then 3 instrumented steps), same GPU lease and library as the bench line",
        "kernel": kern, "dispatches": len(d), "timed_steps_ms": [round(x, 4) for x in timed],
        "timed_mean_ms": round(statistics.mean(timed), 4),
        "timed_median_ms": round(statistics.median(timed), 4),
        "warmup_mean_ms": round(statistics.mean(d[:warm]), 4),
        "instrumented_mean_ms": round(statistics.mean(d[warm + steps:]), 4) if len(d) > warm + steps else None,
        "bench_ms_per_step": b["ms_per_step"], "bench_kernel_ms": r.get("kernel_ms"),
        "step_ideal_ms_spec": ideal,
        "frac_from_profile": round(ideal / statistics.mean(timed), 5) if ideal else None,
        "frac_bench_line": r.get("frac"),
        "library_sha256": hashlib.sha256(open(lib, "rb").read()).hexdigest(),
    }
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps({k: v for k, v in res.items() if k != "timed_steps_ms"}))


if __name__ == "__main__":
    main()
