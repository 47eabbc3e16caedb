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
run def ""
run r72_l40_f16 "" ITR_VIT_RESERVE=72 ITR_VIT_LONG_FRAC=0.40 ITR_FWD_RESERVE=16
run r80_l40_f20 "" ITR_VIT_RESERVE=80 ITR_VIT_LONG_FRAC=0.40 ITR_FWD_RESERVE=20
run r96_l35_f24 "" ITR_VIT_RESERVE=96 ITR_VIT_LONG_FRAC=0.35 ITR_FWD_RESERVE=24
run r64_f24 "" ITR_FWD_RESERVE=24
run r56_l50_f14 "" ITR_VIT_RESERVE=56 ITR_VIT_LONG_FRAC=0.50 ITR_FWD_RESERVE=14
run r64_l50_f20 "" ITR_VIT_LONG_FRAC=0.50 ITR_FWD_RESERVE=20
cat gpurun_out/fvvar.log
