# GPU box: chr10 forward+Viterbi / Viterbi-only / 100 x 100 kbp with the long blocks' Viterbi
# on the 9-wave layout (configuration 9) and on lane groups of three (22), same experiment
# library; then every GPU test + smoke and the bench lines of LINES.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${TAG:-r6c}
ST="c9=ITR_VIT_CFG=9;c22=ITR_VIT_CFG=22"
TAG=$T LIB=itrails_amd/libitrails_hip_exp.so SETTINGS="$ST" REPS=3 BENCH_ARGS="" bash scripts/gpu_envab.sh || exit 1
TAG=$T LIB=itrails_amd/libitrails_hip_exp.so SETTINGS="$ST" REPS=2 BENCH_ARGS="--mode vit" bash scripts/gpu_envab.sh || exit 1
TAG=$T LIB=itrails_amd/libitrails_hip_exp.so SETTINGS="$ST" REPS=2 BENCH_ARGS="--block-len 100000 --steps 5" bash scripts/gpu_envab.sh || exit 1
TAG=$T SKIP_TESTS=$SKIP_TESTS LINES="$LINES" bash scripts/gpu_r6.sh
