# GPU box: every GPU test + smoke, then A/B of the posterior's partitioned forward-store
# launch (lane-group forward tasks; ITR_NO_FWD_GROUPS = the single hybrid launch) and of the
# N = 27 Viterbi layout (ITR_VIT_CFG 0 = four waves, eight lanes per target; 26 = lane groups
# of three on two waves), same experiment library; then the bench lines of LINES.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${TAG:-r6d}
TAG=$T SKIP_TESTS=$SKIP_TESTS LINES= bash scripts/gpu_r6.sh || exit 1
L=itrails_amd/libitrails_hip_exp.so
TAG=$T LIB=$L SETTINGS="fg=;nofg=ITR_NO_FWD_GROUPS=1" REPS=2 BENCH_ARGS="--mode posterior --steps 5" bash scripts/gpu_envab.sh || exit 1
TAG=$T LIB=$L SETTINGS="c0=ITR_VIT_CFG=0;c26=ITR_VIT_CFG=26" REPS=2 BENCH_ARGS="--n-int 3" bash scripts/gpu_envab.sh || exit 1
TAG=$T LIB=$L SETTINGS="c0=ITR_VIT_CFG=0;c26=ITR_VIT_CFG=26" REPS=1 BENCH_ARGS="--n-int 3 --mode vit" bash scripts/gpu_envab.sh || exit 1
TAG=$T LINES="$LINES" bash scripts/gpu_lines.sh
echo done
