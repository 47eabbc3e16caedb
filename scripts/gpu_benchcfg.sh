# GPU box: bench.py under several forced sweep configurations (ITR_SWEEP_CFG), e.g.
#   CFGS="5 12 13" BENCH_ARGS="--mode posterior --n-int 7" bash scripts/gpu_benchcfg.sh
cd $GRAFT_REPO_ROOT
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || exit 1
: > gpurun_out/benchcfg.log
for c in ${CFGS:-auto}; do
  if [ "$c" = auto ]; then unset ITR_SWEEP_CFG; else export ITR_SWEEP_CFG=$c; fi
  timeout -k 10 300 python bench.py --cpu-sample 0 $BENCH_ARGS > gpurun_out/bc.json 2>> gpurun_out/benchcfg.log || exit 1
  python -c "import json;d=json.load(open('gpurun_out/bc.json'));r=d['roofline'];print('cfg $c', round(d['value']/1e6,1),'Mcol/s kernel',r['kernel_ms'],'fwd',r['forward_ms'])" >> gpurun_out/benchcfg.log
done
grep cfg gpurun_out/benchcfg.log
