# model build: optimize-mode bench (config 5 step = rebuild + forward), rocprof kernel stats
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --mode optimize --steps 10 --warmup 2 --verify 0 --host-path 0 --cpu-1core-cols 0 > gpurun_out/bench_opt.json 2> gpurun_out/bench_opt.err || { tail -20 gpurun_out/bench_opt.err; exit 1; }
cat gpurun_out/bench_opt.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/bprof -o bprof --output-format csv -- python scripts/prof_build.py 5 2 > gpurun_out/bprof.log 2>&1 || { tail -20 gpurun_out/bprof.log; exit 1; }
f=$(find gpurun_out/bprof -name '*kernel_stats.csv' | head -1); cp "$f" gpurun_out/build_kernel_stats.csv
python - <<'PY'
import csv
r = list(csv.DictReader(open('gpurun_out/build_kernel_stats.csv')))
tot = sum(float(x['TotalDurationNs']) for x in r)
print('kernel total ms', tot / 1e6, 'launches', sum(int(x['Calls']) for x in r))
for x in r[:16]:
    print(x['Calls'], round(float(x['TotalDurationNs']) / 1e6, 2), round(float(x['AverageNs']) / 1e3, 1), x['Name'][:100])
PY
