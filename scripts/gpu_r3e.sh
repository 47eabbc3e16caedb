# Round 3: build kernel stats (csv), then the fv partition sweep (experiment library)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r3e
O=gpurun_out/r3e
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/bprof -o bprof --output-format csv -- python scripts/prof_build.py 5 2 > $O/bprof.log 2>&1 || { tail -20 $O/bprof.log; exit 1; }
f=$(find $O/bprof -name '*kernel_stats.csv' | head -1); cp "$f" $O/build_kernel_stats.csv
python - <<'PY'
import csv
r = list(csv.DictReader(open('gpurun_out/r3e/build_kernel_stats.csv')))
tot = sum(float(x['TotalDurationNs']) for x in r)
print('kernel total ms', tot / 1e6, 'launches', sum(int(x['Calls']) for x in r))
for x in r[:16]:
    print(x['Calls'], round(float(x['TotalDurationNs']) / 1e6, 2), round(float(x['AverageNs']) / 1e3, 1), x['Name'][:90])
PY
bash scripts/gpu_lab4.sh
