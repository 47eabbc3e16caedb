# GPU box: sweep parity tests, then the default bench twice and the rf=16 variant between them.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_sweeps.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_final.log 2>&1 || { tail -30 gpurun_out/pytest_final.log; exit 1; }
tail -1 gpurun_out/pytest_final.log
: > gpurun_out/final.log
for i in 1 2; do
  timeout -k 10 200 python bench.py --cpu-1core-cols 0 --host-path 0 > gpurun_out/fb.json 2> gpurun_out/fb.err || { tail gpurun_out/fb.err; exit 1; }
  python scripts/bench_line.py gpurun_out/fb.json "rf24_$i" >> gpurun_out/final.log
  ITR_LIB=itrails_amd/libitrails_hip_exp.so ITR_FWD_RESERVE=16 timeout -k 10 200 python bench.py --verify 0 --cpu-1core-cols 0 --host-path 0 > gpurun_out/fb.json 2> gpurun_out/fb.err || { tail gpurun_out/fb.err; exit 1; }
  python scripts/bench_line.py gpurun_out/fb.json "rf16_$i" >> gpurun_out/final.log
done
cat gpurun_out/final.log
