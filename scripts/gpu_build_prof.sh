# model build: instrumented per-call times, then rocprofv3 kernel stats of 2 warm builds
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/prof_build.py 5 2 > gpurun_out/prof_build.log 2>&1 || { tail -20 gpurun_out/prof_build.log; exit 1; }
head -40 gpurun_out/prof_build.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/bprof -o bprof -- python scripts/prof_build.py 5 2 > gpurun_out/bprof.log 2>&1 || { tail -20 gpurun_out/bprof.log; exit 1; }
f=$(find gpurun_out/bprof -name '*kernel_stats.csv' | head -1); cp "$f" gpurun_out/build_kernel_stats.csv
python - <<'PY'
import csv
r = list(csv.DictReader(open('gpurun_out/build_kernel_stats.csv')))
tot = sum(float(x['TotalDurationNs']) for x in r)
print('kernel total ms', tot / 1e6, 'launches', sum(int(x['Calls']) for x in r))
for x in r[:14]:
    print(x['Calls'], round(float(x['TotalDurationNs']) / 1e6, 2), round(float(x['AverageNs']) / 1e3, 1), x['Name'][:90])
PY
