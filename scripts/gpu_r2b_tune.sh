# round 2: hybrid (matrix-core + VALU) sweeps — parity tests, then throughput by urgent share
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
:
:
export ITR_LIB=$PWD/itrails_amd/libitrails_hip_exp.so
: > gpurun_out/r2b.log
for f in ${FRACS:-0.12 0.18 0.25 0.33}; do
  ITR_URGENT_FRAC=$f timeout -k 10 200 python bench.py --steps 10 --warmup 3 --verify 1 --host-path 0 --cpu-1core-cols 0 > gpurun_out/b.json 2>> gpurun_out/r2b.err || { echo "bench FAIL $f"; tail -5 gpurun_out/r2b.err; exit 1; }
  python -c "
import json; d=json.load(open('gpurun_out/b.json')); r=d['roofline']
print('fv frac', $f, 'fwd_ms', r['forward_ms'], 'vit_ms', r['viterbi_ms'], 'value', d['value'], 'relerr', d['loglik_max_rel_err'], d['viterbi_equal'])" >> gpurun_out/r2b.log
done
for f in ${PFRACS:-0.15 0.25 0.35}; do
  ITR_POST_URGENT_FRAC=$f timeout -k 10 300 python bench.py --mode posterior --n-int 7 --steps 3 --warmup 1 --verify 1 --host-path 0 --cpu-1core-cols 0 > gpurun_out/b.json 2>> gpurun_out/r2b.err || { echo "bench FAIL post $f"; tail -5 gpurun_out/r2b.err; exit 1; }
  python -c "
import json; d=json.load(open('gpurun_out/b.json')); r=d['roofline']
print('post7 frac', $f, 'fwd_ms', r['forward_ms'], 'bwd_ms', r['kernel_ms'], 'value', d['value'], d['posterior_allclose_1e-8'], d['row_sum_max_abs_dev_all_columns'])" >> gpurun_out/r2b.log
done
cat gpurun_out/r2b.log
