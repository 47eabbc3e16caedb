"""Per-launch timeline of itr_forward_viterbi calls from a rocprofv3 kernel trace
(rocprofv3 --kernel-trace of bench.py --verify 0): for each call (a run of launches between two fillBuffer/memset groups),
begin / end of every launch relative to the call's first launch, in ms, with its stream
(queue) and grid.  usage: timeline.py <kernel_trace.csv> [calls=2]"""
import csv
import re
import sys


def short(name):
    name = re.sub(r"\(itr::.*$|\(.*$", "", name.replace("void itr::", "")
                  .replace("(anonymous namespace)::", ""))
    return name[:60]


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    ncalls = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    # a call = the launches from 0.1 ms before one bulk launch (role 0 of the mixed / per-wave
    # kernel: the fork) up to 0.1 ms before the next one
    starts = [int(r["Start_Timestamp"]) for r in rows
              if re.search(r"wave_(mixed|vit)_kernel<[^>]*, 0>", r["Kernel_Name"])]
    calls = []
    for i, s0 in enumerate(starts):
        s1 = starts[i + 1] if i + 1 < len(starts) else None
        calls.append([r for r in rows if int(r["Start_Timestamp"]) >= s0 - 100_000 and
                      (s1 is None or int(r["Start_Timestamp"]) < s1 - 100_000) and
                      "fillBuffer" not in r["Kernel_Name"] and "copyBuffer" not in r["Kernel_Name"]
                      and "at::native" not in r["Kernel_Name"]])
    calls = [c for c in calls if any("wave_mixed" in r["Kernel_Name"] for r in c)]
    for c in calls[-ncalls:]:
        t0 = min(int(r["Start_Timestamp"]) for r in c)
        t1 = max(int(r["End_Timestamp"]) for r in c)
        print(f"itr_forward_viterbi call: {(t1 - t0) / 1e6:.3f} ms fork to last kernel end, {len(c)} launches")
        for r in c:
            s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            grid = int(r["Grid_Size_X"]) // max(1, int(r["Workgroup_Size_X"]))
            print(f"  q{r['Queue_Id']:>2} {(s - t0) / 1e6:7.3f} -> {(e - t0) / 1e6:7.3f} "
                  f"({(e - s) / 1e6:6.3f})  wg {grid:5d}  {short(r['Kernel_Name'])}")


if __name__ == "__main__":
    main()
