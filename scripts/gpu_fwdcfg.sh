# Forward-sweep configuration experiment at N = 70 (Viterbi kept on configuration 9).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/fwdcfg.log
for spec in ${SPECS:-20:api 22:api 22:8 23:api}; do
  c=${spec%%:*}; p=${spec##*:}
  if [ "$p" = api ]; then unset ITR_PER_CU; else export ITR_PER_CU=$p; fi
  ITR_SWEEP_CFG=$c ITR_VIT_CFG=9 ITR_VIT_PER_CU=2 timeout -k 10 200 python bench.py --steps 5 --warmup 2 --cpu-sample 0 --check $BARGS > gpurun_out/b.json 2>> gpurun_out/fwdcfg.err || { echo "FAIL $spec"; tail -5 gpurun_out/fwdcfg.err; exit 1; }
  python scripts/bench_line.py gpurun_out/b.json fwd cfg $spec >> gpurun_out/fwdcfg.log
done
cat gpurun_out/fwdcfg.log
