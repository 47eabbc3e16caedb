# Co-scheduling experiment: forward (side stream) beside Viterbi with limited resident
# workgroups per CU for each (prebuilt library).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/conc.log
run() {  # label, then env assignments
  label=$1; shift
  env "$@" timeout -k 10 120 python bench.py --steps 5 --warmup 2 --cpu-sample 0 $BARGS > gpurun_out/b.json 2>> gpurun_out/conc.err || { echo "FAIL $label"; tail -5 gpurun_out/conc.err; exit 1; }
  python scripts/bench_line.py gpurun_out/b.json "$label" >> gpurun_out/conc.log
}
run seq
BARGS="--concurrent 1" run conc_default
BARGS="--concurrent 1" run conc_v1_f1 ITR_VIT_PER_CU=1 ITR_PER_CU=1
BARGS="--concurrent 1" run conc_v1_f2 ITR_VIT_PER_CU=1 ITR_PER_CU=2
BARGS="--concurrent 1" run conc_v1_f3 ITR_VIT_PER_CU=1 ITR_PER_CU=3
BARGS="--concurrent 1" run conc_v2_f1 ITR_VIT_PER_CU=2 ITR_PER_CU=1
BARGS="--concurrent 1" run conc_v20_4_f2 ITR_VIT_CFG=20 ITR_VIT_PER_CU=3 ITR_PER_CU=2
cat gpurun_out/conc.log
