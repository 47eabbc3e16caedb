# GPU box: every GPU test + smoke first (the new layouts' parity), then the A/B of the long
# blocks' Viterbi layout (configuration 9 vs 22) and of the forward's lane-group VALU tasks
# (ITR_NO_FWD_GROUPS), same experiment library; then the bench lines of LINES.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${TAG:-r6c}
O=gpurun_out/$T
mkdir -p $O
TAG=$T SKIP_TESTS=$SKIP_TESTS LINES= bash scripts/gpu_r6.sh || exit 1
X=$PWD/itrails_amd/libitrails_hip_exp.so
ITR_LIB=$X timeout -k 10 200 python scripts/fwd_lone.py > $O/fwd_lone_groups.txt 2>&1 || { tail $O/fwd_lone_groups.txt; exit 1; }
ITR_LIB=$X ITR_NO_FWD_GROUPS=1 timeout -k 10 200 python scripts/fwd_lone.py > $O/fwd_lone_hybrid.txt 2>&1 || { tail $O/fwd_lone_hybrid.txt; exit 1; }
grep forward $O/fwd_lone_*.txt
L=itrails_amd/libitrails_hip_exp.so
ST="c9=ITR_VIT_CFG=9;c22=ITR_VIT_CFG=22;c22nofg=ITR_VIT_CFG=22,ITR_NO_FWD_GROUPS=1"
TAG=$T LIB=$L SETTINGS="$ST" REPS=2 BENCH_ARGS="" bash scripts/gpu_envab.sh || exit 1
TAG=$T LIB=$L SETTINGS="c9=ITR_VIT_CFG=9;c22=ITR_VIT_CFG=22" REPS=2 BENCH_ARGS="--mode vit" bash scripts/gpu_envab.sh || exit 1
TAG=$T LIB=$L SETTINGS="fg=;nofg=ITR_NO_FWD_GROUPS=1" REPS=2 BENCH_ARGS="--mode optimize --steps 10 --warmup 3" bash scripts/gpu_envab.sh || exit 1
TAG=$T LIB=$L SETTINGS="c9=ITR_VIT_CFG=9;c22=ITR_VIT_CFG=22" REPS=1 BENCH_ARGS="--block-len 100000 --steps 5" bash scripts/gpu_envab.sh || exit 1
TAG=$T LINES="$LINES" bash scripts/gpu_lines.sh
echo done
