# Viterbi configuration experiment (prebuilt library): bench throughput for forced Viterbi
# configurations / resident workgroups per CU, on the default and a short-block workload.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/vitcfg.log
SPECS=${SPECS:-"9:api 20:api 20:4 20:6 2:api 2:4"}
for mb in ${MEANS:-2000 300}; do
for spec in $SPECS; do
  c=${spec%%:*}; p=${spec##*:}
  if [ "$p" = api ]; then unset ITR_VIT_PER_CU; else export ITR_VIT_PER_CU=$p; fi
  export ITR_VIT_CFG=$c
  timeout -k 10 120 python bench.py --steps 5 --warmup 2 --cpu-sample 0 --check --mean-block $mb > gpurun_out/b.json 2>> gpurun_out/vitcfg.err || { echo "FAIL $spec"; tail -5 gpurun_out/vitcfg.err; exit 1; }
  python scripts/bench_line.py gpurun_out/b.json mean $mb cfg $spec >> gpurun_out/vitcfg.log
done
done
cat gpurun_out/vitcfg.log
