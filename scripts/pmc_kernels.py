"""Per-kernel sums of rocprofv3 --pmc counter_collection CSVs (every dispatch of a kernel
summed, plus the dispatch count).  usage: python scripts/pmc_kernels.py <csv> [substr]"""
import collections
import csv
import sys


def main():
    rows = csv.DictReader(open(sys.argv[1]))
    sub = sys.argv[2] if len(sys.argv) > 2 else ""
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for r in rows:
        k = r["Kernel_Name"]
        if sub and sub not in k:
            continue
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[k].add(r.get("Dispatch_Id", r.get("Correlation_Id", "")))
    for k, c in sorted(acc.items(), key=lambda kv: -max(kv[1].values())):
        print(k[:90], "dispatches", len(disp[k]))
        for n, v in sorted(c.items()):
            print(f"   {n:32s} {v:.4g}")


if __name__ == "__main__":
    main()
