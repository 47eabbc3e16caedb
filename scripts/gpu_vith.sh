# Viterbi hybrid: parity tests, then the urgent share (experiment library)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_sweeps.py tests/test_gpu_fullsize.py tests/test_gpu_distributed.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_vith.log 2>&1 || { tail -40 gpurun_out/pytest_vith.log; exit 1; }
tail -2 gpurun_out/pytest_vith.log
export ITR_LIB=$PWD/itrails_amd/libitrails_hip_exp.so
: > gpurun_out/vith.log
for f in ${VFRACS:-0.2 0.35 0.5 0.7}; do
  ITR_VIT_URGENT_FRAC=$f timeout -k 10 200 python bench.py --steps 10 --warmup 3 --verify 1 --host-path 0 --cpu-1core-cols 0 > gpurun_out/b.json 2>> gpurun_out/vith.err || { echo "bench FAIL $f"; tail -5 gpurun_out/vith.err; exit 1; }
  python -c "
import json; d=json.load(open('gpurun_out/b.json')); r=d['roofline']
print('vfrac', $f, 'fwd_ms', r['forward_ms'], 'vit_ms', r['viterbi_ms'], 'tb_ms', r['traceback_ms'], 'value', d['value'], d['viterbi_equal'])" >> gpurun_out/vith.log
done
ITR_NO_VITH=1 timeout -k 10 200 python bench.py --steps 10 --warmup 3 --verify 0 --host-path 0 --cpu-1core-cols 0 > gpurun_out/b.json 2>> gpurun_out/vith.err
python -c "
import json; d=json.load(open('gpurun_out/b.json')); r=d['roofline']
print('valu-only vit_ms', r['viterbi_ms'], 'tb_ms', r['traceback_ms'], 'value', d['value'])" >> gpurun_out/vith.log
for f in 0.35; do
  ITR_VIT_URGENT_FRAC=$f timeout -k 10 200 python bench.py --steps 10 --warmup 3 --verify 1 --host-path 0 --cpu-1core-cols 0 --mean-block 300 > gpurun_out/b.json 2>> gpurun_out/vith.err || exit 1
  python -c "
import json; d=json.load(open('gpurun_out/b.json')); r=d['roofline']
print('mean300 vfrac', $f, 'fwd_ms', r['forward_ms'], 'vit_ms', r['viterbi_ms'], 'value', d['value'], d['viterbi_equal'])" >> gpurun_out/vith.log
done
cat gpurun_out/vith.log
