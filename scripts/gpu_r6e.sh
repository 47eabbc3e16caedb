# GPU box: A/B of the (5,5) posterior's split parameters (experiment library: ITR_POST_BFRAC =
# blocks split at least this fraction of the longest, ITR_POST_LO = their split column,
# ITR_POST_URGENT_FRAC = VALU-task threshold), then the bench lines of LINES.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${TAG:-r6e}
L=itrails_amd/libitrails_hip_exp.so
ST="d=;b35=ITR_POST_BFRAC=0.35;b35lo5=ITR_POST_BFRAC=0.35,ITR_POST_LO=0.5;u25=ITR_POST_URGENT_FRAC=0.25,ITR_POST_BFRAC=0.35;u5=ITR_POST_URGENT_FRAC=0.5;lo3=ITR_POST_LO=0.3"
TAG=$T LIB=$L SETTINGS="$ST" REPS=2 BENCH_ARGS="--mode posterior --steps 5" bash scripts/gpu_envab.sh || exit 1
TAG=$T LINES="$LINES" bash scripts/gpu_lines.sh
echo done
