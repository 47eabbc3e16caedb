# Configuration experiment for the other model sizes: posterior at N = 70, forward+Viterbi
# at N = 27 ((3,3)) and N = 46 ((4,4)); ITR_SWEEP_CFG forces every sweep, ITR_VIT_CFG
# Viterbi only (prebuilt library).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/cfgsmall.log
run() {
  label=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps 3 --warmup 1 --cpu-sample 0 $BARGS > gpurun_out/b.json 2>> gpurun_out/cfgsmall.err || { echo "FAIL $label"; tail -5 gpurun_out/cfgsmall.err; exit 1; }
  python scripts/bench_line.py gpurun_out/b.json "$label" >> gpurun_out/cfgsmall.log
}
BARGS="--mode posterior --n-int 5"
run post70_default
for c in 9 15 20 21; do run post70_cfg$c ITR_SWEEP_CFG=$c; done
BARGS="--n-int 3 --check"
run fv27_default
for c in 1 8 14; do run fv27_fwd$c ITR_SWEEP_CFG=$c ITR_VIT_CFG=0; done
for c in 1 8 14; do run fv27_vit$c ITR_VIT_CFG=$c; done
BARGS="--n-int 4 --check"
run fv46_default
for c in 2 8 14 15; do run fv46_fwd$c ITR_SWEEP_CFG=$c ITR_VIT_CFG=1; done
for c in 8 14 15; do run fv46_vit$c ITR_VIT_CFG=$c; done
cat gpurun_out/cfgsmall.log
