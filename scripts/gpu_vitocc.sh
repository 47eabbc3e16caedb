# Viterbi occupancy experiment: library variants with a smaller register budget for the
# one-target-per-lane Viterbi sweep (ITR_VIT_WAVES_PER_SIMD), 2-3 resident workgroups per CU.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/vitocc.log
run() {
  label=$1; shift
  env "$@" timeout -k 10 120 python bench.py --steps 5 --warmup 2 --cpu-sample 0 --check > gpurun_out/b.json 2>> gpurun_out/vitocc.err || { echo "FAIL $label"; tail -5 gpurun_out/vitocc.err; exit 1; }
  python scripts/bench_line.py gpurun_out/b.json "$label" >> gpurun_out/vitocc.log
}
run base
run v8_pc2 ITR_LIB=itrails_amd/libitrails_hip_v8.so ITR_VIT_PER_CU=2
run v8_pc3 ITR_LIB=itrails_amd/libitrails_hip_v8.so ITR_VIT_PER_CU=3
run v7_pc3 ITR_LIB=itrails_amd/libitrails_hip_v7.so ITR_VIT_PER_CU=3
run v8_api ITR_LIB=itrails_amd/libitrails_hip_v8.so
cat gpurun_out/vitocc.log
