# GPU box: balanced long-block set (default) vs none (ITR_VIT_LONG_MIN=1) on chr10 and chr100.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
: > gpurun_out/bal.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_sweeps.py tests/test_gpu_fullsize.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_bal.log 2>&1 || { tail -30 gpurun_out/pytest_bal.log; exit 1; }
tail -1 gpurun_out/pytest_bal.log >> gpurun_out/bal.log
run() { label=$1; bargs=$2; shift 2
  env ITR_LIB=itrails_amd/libitrails_hip_exp.so "$@" timeout -k 10 300 python bench.py --steps 5 --warmup 2 --verify 1 --cpu-1core-cols 0 --host-path 0 $bargs > gpurun_out/c.json 2> gpurun_out/c.err || { echo "FAIL $label" >> gpurun_out/bal.log; cat gpurun_out/bal.log; exit 1; }
  python scripts/bench_line.py gpurun_out/c.json "$label" >> gpurun_out/bal.log; }
run chr10_bal ""
run chr10_nobal "" ITR_VIT_LONG_MIN=1
run chr100_bal "--workload chr100 --steps 3 --warmup 1"
run chr100_nobal "--workload chr100 --steps 3 --warmup 1" ITR_VIT_LONG_MIN=1
run chr10_bal2 ""
cat gpurun_out/bal.log
