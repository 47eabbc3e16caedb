"""Device timeline of warm (n,n) model builds (config 5's rebuild), for a kernel trace:
    rocprofv3 --kernel-trace --output-format csv -d gpurun_out/bt -- python scripts/build_timeline.py run
    python scripts/build_timeline.py analyse <kernel_trace.csv>
`run` performs warm builds separated by 20 ms idle gaps (so the trace splits into builds) and
prints the host wall time of each; `analyse` reports per build the span from the first kernel
to the last, the busy time (union of kernel intervals), and the largest idle gaps with the
kernels either side — where the build waits on the host rather than on the device."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def run(n_int=5, builds=12):
    import torch
    import bench
    from itrails_amd.optimizer import model_for
    names = list(bench.KAT)
    st = {"n_int_AB": n_int, "n_int_ABC": n_int}

    def ev(i):
        x = [bench.KAT[k] * (1.0 + 1e-3 * ((i + j) % 5 - 2)) for j, k in enumerate(names)]
        return model_for(x, names, frozenset(["t_1"]), st)

    for i in range(3):
        ev(i)
    torch.cuda.synchronize()
    for i in range(builds):
        time.sleep(0.02)
        t0 = time.perf_counter()
        ev(10 + i)
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        print(f"build {i}: host return {1e3 * (t1 - t0):.3f} ms, with device {1e3 * (t2 - t0):.3f} ms",
              flush=True)


def analyse(path, top=12):
    import csv
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    builds, cur = [], [rows[0]]
    for r in rows[1:]:
        if r[0] - cur[-1][1] > 10_000_000:  # 10 ms idle: next build
            builds.append(cur)
            cur = []
        cur.append(r)
    builds.append(cur)
    gaps_all = {}
    for bi, b in enumerate(builds):
        span = b[-1][1] - b[0][0]
        busy, end = 0, b[0][0]
        gaps = []
        for s, e, nm in b:
            if s > end:
                gaps.append((s - end, prev_nm if busy else "", nm))
            busy += max(0, e - max(s, end))
            end = max(end, e)
            prev_nm = nm
        ksum = sum(e - s for s, e, _ in b)
        print(f"build {bi}: {len(b)} kernels, span {span / 1e6:.3f} ms, busy {busy / 1e6:.3f} ms, "
              f"kernel sum {ksum / 1e6:.3f} ms, idle {(span - busy) / 1e6:.3f} ms")
        for g, a, c in gaps:
            k = (a[:60], c[:60])
            gaps_all[k] = gaps_all.get(k, 0) + g
    print("largest idle gaps summed over builds (before -> after):")
    for (a, c), g in sorted(gaps_all.items(), key=lambda kv: -kv[1])[:top]:
        print(f"  {g / 1e6 / len(builds):8.3f} ms/build  {a}  ->  {c}")
    tot = {}
    for b in builds:
        for s, e, nm in b:
            tot[nm[:80]] = tot.get(nm[:80], 0) + e - s
    print("kernel time per build:")
    for nm, t in sorted(tot.items(), key=lambda kv: -kv[1])[:20]:
        print(f"  {t / 1e6 / len(builds):8.3f} ms  {nm}")


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run(*(int(a) for a in sys.argv[2:]))
    else:
        analyse(sys.argv[2])
