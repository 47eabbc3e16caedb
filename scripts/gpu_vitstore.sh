# Viterbi store-cost experiment: library variants without the stay-flag / omega-row stores
# (results are wrong by construction: no --check; timing only).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/vitstore.log
run() {
  label=$1; shift
  env "$@" timeout -k 10 120 python bench.py --steps 5 --warmup 2 --cpu-sample 0 $BARGS > gpurun_out/b.json 2>> gpurun_out/vitstore.err || { echo "FAIL $label"; tail -5 gpurun_out/vitstore.err; exit 1; }
  python scripts/bench_line.py gpurun_out/b.json "$label" >> gpurun_out/vitstore.log
}
run base
run nostay ITR_LIB=itrails_amd/libitrails_hip_nostay.so
run noomega ITR_LIB=itrails_amd/libitrails_hip_noomega.so
run nostore ITR_LIB=itrails_amd/libitrails_hip_nostore.so
BARGS="--mean-block 300" run base_m300
BARGS="--mean-block 300" run nostore_m300 ITR_LIB=itrails_amd/libitrails_hip_nostore.so
cat gpurun_out/vitstore.log
