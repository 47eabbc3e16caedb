# Viterbi lane-group hybrid (experiment library): parity, then urgent shares / GL
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
export ITR_LIB=$PWD/itrails_amd/libitrails_hip_exp.so
for h in 1 2; do
ITR_VIT_HYBRID=$h timeout -k 10 300 python -u -m pytest tests/test_gpu_sweeps.py tests/test_gpu_fullsize.py -x -q -m gpu -k "viterbi or Viterbi" --timeout 240 --timeout-method thread > gpurun_out/pytest_vith4.log 2>&1 || { tail -30 gpurun_out/pytest_vith4.log; exit 1; }
tail -1 gpurun_out/pytest_vith4.log
done
: > gpurun_out/vith4.log
run() {
  lab=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps 10 --warmup 3 --verify 1 --host-path 0 --cpu-1core-cols 0 > gpurun_out/b.json 2>> gpurun_out/vith4.err || { echo "bench FAIL $lab"; tail -5 gpurun_out/vith4.err; exit 1; }
  python -c "
import json; d=json.load(open('gpurun_out/b.json')); r=d['roofline']
print('$lab', 'vit_ms', r['viterbi_ms'], 'value', d['value'], d['viterbi_equal'])" >> gpurun_out/vith4.log
}
run base ITR_X=0 || exit 1
for f in 0.3 0.5 0.7; do
  run "gl4_$f" ITR_VIT_HYBRID=1 ITR_VIT_URGENT_FRAC=$f || exit 1
  run "gl2_$f" ITR_VIT_HYBRID=2 ITR_VIT_URGENT_FRAC=$f || exit 1
done
run "gl2_pc2_0.5" ITR_VIT_HYBRID=2 ITR_VIT_PER_CU=2 ITR_VIT_URGENT_FRAC=0.5 || exit 1
cat gpurun_out/vith4.log
