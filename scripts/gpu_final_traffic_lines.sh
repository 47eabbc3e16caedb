# GPU box, after the final pass's profiles are copied under profiles/: the lines whose
# roofline carries this build's PMC traffic (chr10 forward + Viterbi, Viterbi, RCCL world 1,
# posteriors, config 5 three times), outputs under gpurun_out/$TAG.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${TAG:-r6y2}
B="--cpu-1core-cols 0 --host-path 0"
TAG=$T LINES="fv:;vit:$B --mode vit;rccl1:$B --dist 1 --backend nccl;post77:$B --mode posterior --n-int 7 --steps 5;post55:$B --mode posterior --n-int 5 --steps 5;opt55:$B --mode optimize --steps 10 --warmup 3;opt55b:$B --mode optimize --steps 10 --warmup 3;opt55c:$B --mode optimize --steps 10 --warmup 3" bash scripts/gpu_lines.sh
