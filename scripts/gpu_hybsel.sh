# hybrid vs VALU-only by model size (experiment library)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
export ITR_LIB=$PWD/itrails_amd/libitrails_hip_exp.so
: > gpurun_out/hybsel.log
one() {  # tag env... -- bench args
  tag=$1; shift
  timeout -k 10 300 env "$@" --host-path 0 --cpu-1core-cols 0 --verify 1 > gpurun_out/b.json 2>> gpurun_out/hybsel.err || { echo "FAIL $tag"; tail -5 gpurun_out/hybsel.err; exit 1; }
  python -c "
import json; d=json.load(open('gpurun_out/b.json')); r=d['roofline']
print('$tag', 'fwd_ms', r['forward_ms'], 'kernel_ms', r['kernel_ms'], 'value', d['value'], 'ok', d.get('viterbi_equal', d.get('posterior_allclose_1e-8')))" >> gpurun_out/hybsel.log
}
one post5_valu ITR_NO_MFMA=1 python bench.py --mode posterior --n-int 5 --steps 5 --warmup 2
one post5_hyb ITR_HYB_POST=1 python bench.py --mode posterior --n-int 5 --steps 5 --warmup 2
one int5_valu ITR_NO_MFMA=1 python bench.py --model introgression --n-int 5 --steps 5 --warmup 2
one int5_hyb X=1 python bench.py --model introgression --n-int 5 --steps 5 --warmup 2
one kat4_valu ITR_NO_MFMA=1 python bench.py --n-int 4 --steps 5 --warmup 2
one kat4_hyb X=1 python bench.py --n-int 4 --steps 5 --warmup 2
one int5post_valu ITR_NO_MFMA=1 python bench.py --mode posterior --model introgression --n-int 5 --steps 3 --warmup 1
one int5post_hyb ITR_HYB_POST=1 python bench.py --mode posterior --model introgression --n-int 5 --steps 3 --warmup 1
cat gpurun_out/hybsel.log
