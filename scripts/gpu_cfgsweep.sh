# Sweep-kernel configuration experiment: per-step cycles (diag build) and bench throughput
# for forced configurations / resident-workgroup counts.
cd $GRAFT_REPO_ROOT
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || exit 1
python -c "from itrails_amd.build import build; build(force=True, diag=True)" >> gpurun_out/build.log 2>&1 || exit 1
: > gpurun_out/cfgsweep.log
CFGS=${CFGS:-"2:api 2:2 2:3 7:api 7:3 7:4"}
for spec in $CFGS; do
  c=${spec%%:*}; p=${spec##*:}
  if [ "$p" = api ]; then unset ITR_PER_CU; else export ITR_PER_CU=$p; fi
  export ITR_SWEEP_CFG=$c
  timeout -k 10 200 python scripts/diag_probe.py >> gpurun_out/cfgsweep.log 2>&1 || exit 1
  timeout -k 10 200 python bench.py --steps 5 --warmup 2 --cpu-sample 0 > gpurun_out/b.json 2>> gpurun_out/cfgsweep.log || exit 1
  python -c "import json;d=json.load(open('gpurun_out/b.json'));r=d['roofline'];print('$spec','BENCH',round(d['value']/1e6,1),'Mcol/s fwd',r['forward_ms'],'vit',r['kernel_ms'])" >> gpurun_out/cfgsweep.log
done
cat gpurun_out/cfgsweep.log | grep -v amdgpu.ids
