cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
export ITR_LIB=$PWD/itrails_amd/libitrails_hip_exp.so
: > gpurun_out/vcfg.log
for c in 9 15 16 14 18 19 8; do
  ITR_VIT_CFG=$c timeout -k 10 200 python bench.py --steps 8 --warmup 2 --verify 1 --host-path 0 --cpu-1core-cols 0 > gpurun_out/b.json 2>> gpurun_out/vcfg.err || { echo "bench FAIL $c"; tail -5 gpurun_out/vcfg.err; exit 1; }
  python -c "
import json; d=json.load(open('gpurun_out/b.json')); r=d['roofline']
print('cfg $c', 'vit_ms', r['viterbi_ms'], 'tb_ms', r['traceback_ms'], d['viterbi_equal'])" >> gpurun_out/vcfg.log
done
cat gpurun_out/vcfg.log
