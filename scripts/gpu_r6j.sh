# GPU box: scripts/gpu_r6i.sh (tests + the forward-store lane-group A/B), then
# scripts/gpu_r6h.sh (N = 95 / 133 Viterbi layouts, the hybrid posterior at N = 95).
cd $GRAFT_REPO_ROOT
TAG=${TAG:-r6j} bash scripts/gpu_r6i.sh || exit 1
TAG=${TAG:-r6j} bash scripts/gpu_r6h.sh
