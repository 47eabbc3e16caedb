cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
: > gpurun_out/dbgwave.log
for L in 20 100,7,300,2000 3000,20,30,40 5000,4000,3000,2000,1000,999,17,16,15,1,0,2; do
  echo "== $L" >> gpurun_out/dbgwave.log
  timeout -k 5 30 python -u scripts/dbg_wave.py 70 $L >> gpurun_out/dbgwave.log 2>&1 || { echo "FAIL rc=$? $L" >> gpurun_out/dbgwave.log; cat gpurun_out/dbgwave.log; exit 1; }
done
cat gpurun_out/dbgwave.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_sweeps.py tests/test_gpu_fullsize.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_wave.log 2>&1 || { tail -40 gpurun_out/pytest_wave.log; exit 1; }
tail -2 gpurun_out/pytest_wave.log
timeout -k 10 400 python bench.py --cpu-1core-cols 0 --host-path 0 > gpurun_out/bench_wave.json 2> gpurun_out/bench_wave.err || { tail gpurun_out/bench_wave.err; exit 1; }
python scripts/bench_line.py gpurun_out/bench_wave.json wave
