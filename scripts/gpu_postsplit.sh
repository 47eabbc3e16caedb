cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_gpu_sweeps.py tests/test_gpu_fullsize.py tests/test_gpu_distributed.py tests/test_gpu_model.py tests/test_gpu_dense.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_ps.log 2>&1 || { tail -40 gpurun_out/pytest_ps.log; exit 1; }
tail -2 gpurun_out/pytest_ps.log
timeout -k 10 300 python scripts/dbg_post.py > gpurun_out/dbg_post.log 2>&1 || { tail -20 gpurun_out/dbg_post.log; exit 1; }
grep -v amdgpu.ids gpurun_out/dbg_post.log
: > gpurun_out/ps.log
run() {
  lab=$1; shift
  timeout -k 10 300 python bench.py --steps 3 --warmup 1 --verify 1 --host-path 0 --cpu-1core-cols 0 "$@" > gpurun_out/b_$lab.json 2>> gpurun_out/ps.err || { echo "bench FAIL $lab"; tail -5 gpurun_out/ps.err; exit 1; }
  python -c "
import json; d=json.load(open('gpurun_out/b_$lab.json')); r=d['roofline']
print('$lab', d['value'], 'fwd', r.get('forward_ms'), 'bwd/vit', r.get('viterbi_ms'), 'kern', r.get('kernel_ms'), d.get('viterbi_equal'), d.get('loglik_max_rel_err'))" >> gpurun_out/ps.log
}
run long_fv --block-len 100000 || exit 1
run long_post --block-len 100000 --mode posterior || exit 1
run chr10_post --mode posterior || exit 1
run chr10_fv || exit 1
cat gpurun_out/ps.log
