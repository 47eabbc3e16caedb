# (7,7) posterior: one vs two matrix-core groups per workgroup, by urgent share
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
export ITR_LIB=$PWD/itrails_amd/libitrails_hip_exp.so
: > gpurun_out/p133.log
for spec in ${SPECS:-5:0.2 5:0.35 5:0.5 5:0.7 7:0.35}; do
  c=${spec%%:*}; f=${spec##*:}
  ITR_MCFG=$c ITR_POST_URGENT_FRAC=$f timeout -k 10 300 python bench.py --mode posterior --n-int 7 --steps 3 --warmup 1 --verify 1 --host-path 0 --cpu-1core-cols 0 > gpurun_out/b.json 2>> gpurun_out/p133.err || { echo "FAIL $spec"; tail -5 gpurun_out/p133.err; exit 1; }
  python -c "
import json; d=json.load(open('gpurun_out/b.json')); r=d['roofline']
print('post7 cfg $c frac $f fwd_ms', r['forward_ms'], 'bwd_ms', r['kernel_ms'], 'value', d['value'], d['posterior_allclose_1e-8'])" >> gpurun_out/p133.log
done
cat gpurun_out/p133.log
