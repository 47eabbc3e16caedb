# Sweep configuration probe (experiment library, env knobs): lone-block step latency and
# bulk throughput (short blocks, no long tail) per configuration index.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
export ITR_LIB=$PWD/itrails_amd/libitrails_hip_exp.so
: > gpurun_out/cfgprobe.log
for c in ${LATCFGS:-9 14 15 16 17 18 19 20 2 3}; do
  ITR_SWEEP_CFG=$c timeout -k 10 60 python scripts/lat1.py >> gpurun_out/cfgprobe.log 2>> gpurun_out/cfgprobe.err || { echo "lat FAIL $c"; tail -5 gpurun_out/cfgprobe.err; exit 1; }
done
for mb in ${MEANS:-300 2000}; do
for spec in ${SPECS:-9:api 15:api 15:3 15:4 14:api 16:api 20:api}; do
  c=${spec%%:*}; p=${spec##*:}
  if [ "$p" = api ]; then unset ITR_PER_CU; else export ITR_PER_CU=$p; fi
  ITR_SWEEP_CFG=$c timeout -k 10 120 python bench.py --steps 5 --warmup 2 --verify 0 --host-path 0 --cpu-1core-cols 0 --mean-block $mb > gpurun_out/b.json 2>> gpurun_out/cfgprobe.err || { echo "bench FAIL $spec"; tail -5 gpurun_out/cfgprobe.err; exit 1; }
  python -c "
import json,sys; d=json.load(open('gpurun_out/b.json')); r=d['roofline']
print('mean', $mb, 'cfg', '$spec', 'fwd_ms', r['forward_ms'], 'vit_ms', r['viterbi_ms'], 'tb_ms', r['traceback_ms'], 'value', d['value'])" >> gpurun_out/cfgprobe.log
done
done
cat gpurun_out/cfgprobe.log
