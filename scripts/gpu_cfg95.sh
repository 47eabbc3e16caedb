# N = 95 (introgression (5,5) model) configuration experiment, Viterbi and forward forced
# separately (prebuilt library).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/cfg95.log
B="python bench.py --model introgression --mode fv --n-int 5 --steps 3 --warmup 1 --cpu-sample 0"
for c in 4 10 12 16 18; do
  ITR_VIT_CFG=$c timeout -k 10 200 $B --check > gpurun_out/b.json 2>> gpurun_out/cfg95.err || { echo "FAIL vit $c"; tail -5 gpurun_out/cfg95.err; exit 1; }
  python scripts/bench_line.py gpurun_out/b.json vitcfg $c >> gpurun_out/cfg95.log
done
for c in 4 12 16 18; do
  ITR_SWEEP_CFG=$c ITR_VIT_CFG=4 timeout -k 10 200 $B > gpurun_out/b.json 2>> gpurun_out/cfg95.err || { echo "FAIL fwd $c"; tail -5 gpurun_out/cfg95.err; exit 1; }
  python scripts/bench_line.py gpurun_out/b.json fwdcfg $c >> gpurun_out/cfg95.log
done
cat gpurun_out/cfg95.log
