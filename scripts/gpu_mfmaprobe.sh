# matrix-core sweep probe (experiment library): all-MFMA bulk throughput on short blocks by
# resident workgroups per CU, and the hybrid at the default workload by urgent share
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
export ITR_LIB=$PWD/itrails_amd/libitrails_hip_exp.so
: > gpurun_out/mprobe.log
run() {  # label, env..., -- bench args
  timeout -k 10 200 env "$@" > gpurun_out/b.json 2>> gpurun_out/mprobe.err || { echo "FAIL $*"; tail -5 gpurun_out/mprobe.err; exit 1; }
}
for pc in 1 2 3; do
  ITR_SPLIT_FRAC=0 ITR_URGENT_FRAC=9 ITR_HYB_PER_CU=$pc timeout -k 10 200 python bench.py --steps 10 --warmup 3 --verify 1 --host-path 0 --cpu-1core-cols 0 --mean-block 300 > gpurun_out/b.json 2>> gpurun_out/mprobe.err || { echo FAIL; tail -5 gpurun_out/mprobe.err; exit 1; }
  python -c "
import json; d=json.load(open('gpurun_out/b.json')); r=d['roofline']
print('allmfma mean300 per_cu $pc fwd_ms', r['forward_ms'], 'relerr', d['loglik_max_rel_err'])" >> gpurun_out/mprobe.log
done
for pc in 2 3; do
  ITR_SPLIT_FRAC=0 ITR_URGENT_FRAC=9 ITR_HYB_PER_CU=$pc timeout -k 10 300 python bench.py --mode posterior --n-int 7 --steps 3 --warmup 1 --verify 0 --host-path 0 --cpu-1core-cols 0 --mean-block 300 > gpurun_out/b.json 2>> gpurun_out/mprobe.err || { echo FAIL; tail -5 gpurun_out/mprobe.err; exit 1; }
  python -c "
import json; d=json.load(open('gpurun_out/b.json')); r=d['roofline']
print('allmfma post7 mean300 per_cu $pc fwd_ms', r['forward_ms'], 'bwd_ms', r['kernel_ms'])" >> gpurun_out/mprobe.log
done
ITR_SWEEP_CFG=20 timeout -k 10 200 python bench.py --steps 10 --warmup 3 --verify 0 --host-path 0 --cpu-1core-cols 0 --mean-block 300 --n-int 4 > gpurun_out/b.json 2>> gpurun_out/mprobe.err
python -c "
import json; d=json.load(open('gpurun_out/b.json')); r=d['roofline']
print('n-int 4 (N=46) mean300 fwd_ms', r['forward_ms'])" >> gpurun_out/mprobe.log
cat gpurun_out/mprobe.log
