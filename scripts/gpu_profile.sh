# GPU box: build, GPU tests, bench, rocprofv3 kernel-trace stats and separate PMC passes
# (FETCH_SIZE and WRITE_SIZE each in their own run, no trace domains).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${TAG:-r1}
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || { echo BUILD FAIL; tail -20 gpurun_out/build.log; exit 1; }
timeout -k 10 900 python -m pytest tests -x -q -m gpu --timeout=300 --timeout-method=thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 300 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || { tail gpurun_out/bench_default.err; exit 1; }
cat gpurun_out/bench_default.json
B="python3 bench.py --steps 3 --warmup 1 --cpu-sample 0"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o trace --output-format csv -- $B > gpurun_out/prof_trace.log 2>&1 || { tail gpurun_out/prof_trace.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/prof_$TAG -o pmc_fetch --output-format csv -- $B > gpurun_out/prof_fetch.log 2>&1 || { tail gpurun_out/prof_fetch.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/prof_$TAG -o pmc_write --output-format csv -- $B > gpurun_out/prof_write.log 2>&1 || { tail gpurun_out/prof_write.log; exit 1; }
find gpurun_out/prof_$TAG -name "*.csv" | head -20
