"""Kernel timeline of the last posterior call in a rocprofv3 kernel trace: start / end of
every kernel launched after the last forward-store launch, relative to its start, with the
queue each ran on and its grid.  usage: post_timeline.py <kernel_trace.csv> (a rocprofv3
--kernel-trace of bench.py --mode posterior)."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
fw = [i for i, r in enumerate(rows) if "hybrid_sweep_kernel" in r["Kernel_Name"] and ", 1, 1, 2," in r["Kernel_Name"]]
if not fw:
    sys.exit("no forward-store hybrid launch")
i0 = fw[-1]
# include the beta launch dispatched just before it
start = max(0, i0 - 4)
t0 = int(rows[i0]["Start_Timestamp"])
for r in rows[start:]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    print(f"q{r['Queue_Id']:>3} grid {int(r['Grid_Size_X']) // int(r['Workgroup_Size_X']):5d}  "
          f"{(s - t0) / 1e6:8.3f} -> {(e - t0) / 1e6:8.3f} ms  {r['Kernel_Name'][:90]}")
