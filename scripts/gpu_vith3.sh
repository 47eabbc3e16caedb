# QL=4 Viterbi hybrid at 5 waves/SIMD (experiment library)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
export ITR_LIB=$PWD/itrails_amd/libitrails_hip_exp.so
: > gpurun_out/vith3.log
run() {  # label, env...
  lab=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps 10 --warmup 3 --verify 1 --host-path 0 --cpu-1core-cols 0 > gpurun_out/b.json 2>> gpurun_out/vith3.err || { echo "bench FAIL $lab"; tail -5 gpurun_out/vith3.err; exit 1; }
  python -c "
import json; d=json.load(open('gpurun_out/b.json')); r=d['roofline']
print('$lab', 'vit_ms', r['viterbi_ms'], 'value', d['value'], d['viterbi_equal'])" >> gpurun_out/vith3.log
}
for f in 0.25 0.5; do
  run "ql4_wait_$f" ITR_VIT_HYBRID=1 ITR_VIT_URGENT_FRAC=$f || exit 1
  run "ql4_nocu_$f" ITR_VIT_HYBRID=1 ITR_VIT_NOCU=1 ITR_VIT_URGENT_FRAC=$f || exit 1
done
cat gpurun_out/vith3.log
