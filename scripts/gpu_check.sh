# GPU box: build, run the GPU test-suite, a short bench, then a rocprofv3 kernel trace
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || { echo BUILD FAIL; tail -20 gpurun_out/build.log; exit 1; }
timeout -k 10 900 python -m pytest tests -x -q -m gpu --timeout=300 --timeout-method=thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -30 gpurun_out/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --check ${BENCH_ARGS} > gpurun_out/bench1.json 2> gpurun_out/bench1.err; rc=$?
cat gpurun_out/bench1.json; tail -5 gpurun_out/bench1.err
[ $rc -ne 0 ] && exit $rc
if [ -n "$PROFILE" ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --cpu-sample 0 > gpurun_out/prof.log 2>&1; rc=$?
  tail -3 gpurun_out/prof.log
fi
exit $rc
