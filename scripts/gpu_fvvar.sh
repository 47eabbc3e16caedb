# GPU box: run-to-run and step-to-step variation of the combined forward+Viterbi step.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
: > gpurun_out/fvvar.log
run() {  # label, bench args, then env assignments
  label=$1; bargs=$2; shift 2
  env ITR_LIB=itrails_amd/libitrails_hip_exp.so "$@" timeout -k 10 120 python bench.py --steps 12 --warmup 2 --verify 0 --cpu-1core-cols 0 --host-path 0 $bargs > gpurun_out/ws.json 2> gpurun_out/ws.err || { echo "FAIL $label" >> gpurun_out/fvvar.log; cat gpurun_out/fvvar.log; exit 1; }
  python scripts/bench_line.py gpurun_out/ws.json "$label" >> gpurun_out/fvvar.log
  grep "^step" gpurun_out/ws.err | tr '\n' ' ' >> gpurun_out/fvvar.log; echo >> gpurun_out/fvvar.log
}
run side ""
run side_sync "" BENCH_STEP_TIMES=1
run dflt "--stream default"
run side_q8 "" GPU_MAX_HW_QUEUES=8
run q8_beside1 "" GPU_MAX_HW_QUEUES=8 ITR_FV_BESIDE=1
run q8_beside2 "" GPU_MAX_HW_QUEUES=8 ITR_FV_BESIDE=2
run old "--overlap 0" ITR_NO_WAVE=1
cat gpurun_out/fvvar.log
