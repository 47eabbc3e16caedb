# GPU box: wave Viterbi (side-stream long blocks + per-wave sweep): parity, then configurations.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
: > gpurun_out/wavesweep.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_sweeps.py tests/test_gpu_fullsize.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_wave.log 2>&1 || { tail -40 gpurun_out/pytest_wave.log; exit 1; }
tail -2 gpurun_out/pytest_wave.log
run() {  # label, bench args, then env assignments
  label=$1; bargs=$2; shift 2
  env ITR_LIB=itrails_amd/libitrails_hip_exp.so "$@" timeout -k 10 120 python bench.py --steps 5 --warmup 2 --verify 1 --cpu-1core-cols 0 --host-path 0 $bargs > gpurun_out/ws.json 2>> gpurun_out/ws.err || { echo "FAIL $label" >> gpurun_out/wavesweep.log; cat gpurun_out/wavesweep.log; exit 1; }
  python scripts/bench_line.py gpurun_out/ws.json "$label" >> gpurun_out/wavesweep.log
}
run old "--overlap 0" ITR_NO_WAVE=1
run wfwd ""
run wfwd_r48 "" ITR_VIT_RESERVE=48
run wfwd_r80 "" ITR_VIT_RESERVE=80
run hyb "" ITR_FV_HYBRID=1
run lb "--block-len 100000"
run short "--mean-block 300"
cat gpurun_out/wavesweep.log
