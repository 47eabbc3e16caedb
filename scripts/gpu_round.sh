# GPU box: GPU tests (prebuilt in-tree .so), smoke, default bench, rocprofv3 kernel stats and
# separate FETCH_SIZE / WRITE_SIZE PMC passes of a short bench run. Every GPU step is
# time-limited; stop at the first failure.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${TAG:-r2}
mkdir -p gpurun_out
if [ -z "$SKIP_TESTS" ]; then
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1 || { tail -30 gpurun_out/pytest_gpu_$TAG.log; exit 1; }
tail -2 gpurun_out/pytest_gpu_$TAG.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || { tail -20 gpurun_out/smoke_$TAG.log; exit 1; }
tail -1 gpurun_out/smoke_$TAG.log
fi
timeout -k 10 400 python bench.py $BENCH_ARGS > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail gpurun_out/bench_$TAG.err; exit 1; }
cat gpurun_out/bench_$TAG.json
B="python3 bench.py --steps 3 --warmup 1 --verify 0 --cpu-1core-cols 0 --host-path 0 $BENCH_ARGS"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o trace --output-format csv -- $B > gpurun_out/prof_trace_$TAG.log 2>&1 || { tail gpurun_out/prof_trace_$TAG.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/prof_$TAG -o pmc_fetch --output-format csv -- $B > gpurun_out/prof_fetch_$TAG.log 2>&1 || { tail gpurun_out/prof_fetch_$TAG.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/prof_$TAG -o pmc_write --output-format csv -- $B > gpurun_out/prof_write_$TAG.log 2>&1 || { tail gpurun_out/prof_write_$TAG.log; exit 1; }
find gpurun_out/prof_$TAG -name "*stats.csv" -o -name "*counter_collection.csv"
