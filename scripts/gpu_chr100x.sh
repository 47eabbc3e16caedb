# GPU box: chr100 combined-call variants (experiment library).
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
: > gpurun_out/c100.log
run() { label=$1; shift
  env ITR_LIB=itrails_amd/libitrails_hip_exp.so "$@" timeout -k 10 300 python bench.py --workload chr100 --steps 3 --warmup 1 --verify 0 --cpu-1core-cols 0 --host-path 0 > gpurun_out/c.json 2> gpurun_out/c.err || { echo "FAIL $label" >> gpurun_out/c100.log; cat gpurun_out/c100.log; exit 1; }
  python scripts/bench_line.py gpurun_out/c.json "$label" >> gpurun_out/c100.log; }
run splitall ITR_FV_SPLIT_CAP=100000
run splitall_f32 ITR_FV_SPLIT_CAP=100000 ITR_FWD_RESERVE=32
run r96 ITR_VIT_RESERVE=96
run r96_splitall ITR_VIT_RESERVE=96 ITR_FV_SPLIT_CAP=100000 ITR_FWD_RESERVE=40
cat gpurun_out/c100.log
