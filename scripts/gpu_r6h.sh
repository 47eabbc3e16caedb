# GPU box: Viterbi layout A/B at N = 95 (configuration 16 = six waves x four lanes, 3 = four
# waves x three targets per lane, 18 = three waves x two targets, four lanes) and N = 133
# (23 = lane groups of five, 21 = six waves x three targets per lane), the hybrid posterior at
# N = 95 (ITR_HYB_POST) with the (5,5) split constants; experiment library.  Then the
# final pass's other lines (LINES).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${TAG:-r6h}
L=itrails_amd/libitrails_hip_exp.so
TAG=$T LIB=$L SETTINGS="c16=ITR_VIT_CFG=16;c3=ITR_VIT_CFG=3;c18=ITR_VIT_CFG=18" REPS=2 BENCH_ARGS="--model introgression --mode vit --steps 10" bash scripts/gpu_envab.sh || exit 1
TAG=$T LIB=$L SETTINGS="c23=ITR_VIT_CFG=23;c21=ITR_VIT_CFG=21" REPS=1 BENCH_ARGS="--n-int 7 --mode vit --steps 5" bash scripts/gpu_envab.sh || exit 1
TAG=$T LIB=$L SETTINGS="valu=;hyb=ITR_HYB_POST=1;hyb25=ITR_HYB_POST=1,ITR_POST_URGENT_FRAC=0.25,ITR_POST_BFRAC=0.25" REPS=2 BENCH_ARGS="--model introgression --mode posterior --steps 5" bash scripts/gpu_envab.sh || exit 1
[ -n "$LINES" ] && TAG=$T LINES="$LINES" bash scripts/gpu_lines.sh
echo done
