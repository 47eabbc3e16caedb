# Sweep-kernel configuration experiment (bench throughput only): forced configuration
# (ITR_SWEEP_CFG, applies to every sweep mode) and resident workgroups per CU (ITR_PER_CU).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
: > gpurun_out/cfgbench.log
CFGS=${CFGS:-"2:api 9:api"}
MODE=${MODE:-fv}
for spec in $CFGS; do
  c=${spec%%:*}; p=${spec##*:}
  if [ "$p" = api ]; then unset ITR_PER_CU; else export ITR_PER_CU=$p; fi
  export ITR_SWEEP_CFG=$c
  timeout -k 10 200 python bench.py --steps 5 --warmup 2 --cpu-sample 0 --mode $MODE ${BENCH_ARGS} > gpurun_out/b.json 2>> gpurun_out/cfgbench.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/b.json'));r=d['roofline'];print('$spec','BENCH',round(d['value']/1e6,1),'Mcol/s fwd',r['forward_ms'],'k2',r['kernel_ms'],'tb',r['traceback_ms'])" >> gpurun_out/cfgbench.log
done
cat gpurun_out/cfgbench.log
