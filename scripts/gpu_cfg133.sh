# N = 133 ((7,7) model) configuration experiment: posterior (config 3) and forward+Viterbi
# for forced sweep configurations (prebuilt library).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/cfg133.log
for c in ${CFGS:-5 12 13 17 21}; do
  ITR_SWEEP_CFG=$c timeout -k 10 200 python bench.py --mode posterior --n-int 7 --steps 3 --warmup 1 --cpu-sample 0 > gpurun_out/b.json 2>> gpurun_out/cfg133.err || { echo "FAIL post $c"; tail -5 gpurun_out/cfg133.err; exit 1; }
  python scripts/bench_line.py gpurun_out/b.json posterior cfg $c >> gpurun_out/cfg133.log
done
for c in ${CFGS:-5 12 13 17 21}; do
  ITR_SWEEP_CFG=$c timeout -k 10 200 python bench.py --mode fv --n-int 7 --steps 3 --warmup 1 --cpu-sample 0 --check > gpurun_out/b.json 2>> gpurun_out/cfg133.err || { echo "FAIL fv $c"; tail -5 gpurun_out/cfg133.err; exit 1; }
  python scripts/bench_line.py gpurun_out/b.json fv cfg $c >> gpurun_out/cfg133.log
done
cat gpurun_out/cfg133.log
