# Viterbi: CU-exclusive long blocks (experiment library), urgent fractions
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
export ITR_LIB=$PWD/itrails_amd/libitrails_hip_exp.so
ITR_VIT_EXCL_FRAC=0.5 timeout -k 10 300 python -u -m pytest tests/test_gpu_sweeps.py tests/test_gpu_fullsize.py -x -q -m gpu -k "viterbi or Viterbi" --timeout 240 --timeout-method thread > gpurun_out/pytest_excl.log 2>&1 || { tail -30 gpurun_out/pytest_excl.log; exit 1; }
tail -1 gpurun_out/pytest_excl.log
: > gpurun_out/excl.log
run() {
  lab=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps 10 --warmup 3 --verify 1 --host-path 0 --cpu-1core-cols 0 > gpurun_out/b.json 2>> gpurun_out/excl.err || { echo "bench FAIL $lab"; tail -5 gpurun_out/excl.err; exit 1; }
  python -c "
import json; d=json.load(open('gpurun_out/b.json')); r=d['roofline']
print('$lab', 'vit_ms', r['viterbi_ms'], 'fwd_ms', r['forward_ms'], 'value', d['value'], d['viterbi_equal'])" >> gpurun_out/excl.log
}
run base ITR_X=0 || exit 1
for f in 0.8 0.6 0.4 0.25; do run "excl_$f" ITR_VIT_EXCL_FRAC=$f || exit 1; done
run mean300_base ITR_X=0 || exit 1
cat gpurun_out/excl.log
unset ITR_LIB
timeout -k 10 400 python -u -m pytest tests/test_gpu_dense.py tests/test_gpu_model.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_build2.log 2>&1 || { tail -40 gpurun_out/pytest_build2.log; exit 1; }
tail -1 gpurun_out/pytest_build2.log
timeout -k 10 300 python -u scripts/prof_build.py 5 3 > gpurun_out/prof_build.log 2>&1 || { tail -20 gpurun_out/prof_build.log; exit 1; }
head -16 gpurun_out/prof_build.log
