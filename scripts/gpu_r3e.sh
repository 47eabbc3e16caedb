# Round 3: build kernel stats (csv), then the fv partition sweep (experiment library)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r3e
O=gpurun_out/r3e
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_dense.py tests/test_gpu_model.py tests/test_gpu_distributed.py -k "vanloan or model or split" > $O/model.log 2>&1 || { tail -30 $O/model.log; exit 1; }
tail -2 $O/model.log
timeout -k 10 300 python -u scripts/prof_build.py 5 3 > $O/prof_build.log 2>&1 || { tail -20 $O/prof_build.log; exit 1; }
head -8 $O/prof_build.log
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
