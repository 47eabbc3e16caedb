# GPU box: lone-step and N = 95 / 133 Viterbi A/B of the lane-group layouts against the
# previous configurations (same experiment library, ITR_VIT_CFG), every GPU test + smoke, then
# the bench lines of LINES; outputs under gpurun_out/$TAG.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r6b}
mkdir -p $O
X=$PWD/itrails_amd/libitrails_hip_exp.so
for T in 18377 100000; do
  for c in 9 22; do
    ITR_LIB=$X ITR_VIT_CFG=$c timeout -k 10 120 python scripts/vit_lone.py $T 1 >> $O/lone.txt 2>&1 || { tail $O/lone.txt; exit 1; }
  done
done
cat $O/lone.txt
B="--cpu-1core-cols 0 --host-path 0 --verify 0 --steps 5 --warmup 2 --mode vit"
for c in 17 23 25; do
  ITR_LIB=$X ITR_VIT_CFG=$c timeout -k 10 200 python bench.py $B --n-int 7 > $O/vit77_cfg$c.json 2> $O/vit77_cfg$c.err || { tail $O/vit77_cfg$c.err; exit 1; }
  python scripts/bench_line.py $O/vit77_cfg$c.json vit77 cfg$c
done
for c in 16 24; do
  ITR_LIB=$X ITR_VIT_CFG=$c timeout -k 10 200 python bench.py $B --model introgression > $O/vitint_cfg$c.json 2> $O/vitint_cfg$c.err || { tail $O/vitint_cfg$c.err; exit 1; }
  python scripts/bench_line.py $O/vitint_cfg$c.json vitint cfg$c
done
TAG=${TAG:-r6b} SKIP_TESTS=$SKIP_TESTS LINES="$LINES" bash scripts/gpu_r6.sh
