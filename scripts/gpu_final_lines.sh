# GPU box, round 6 final pass, second part: every other BASELINE line on the same library.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${TAG:-r6z}
B="--cpu-1core-cols 0 --host-path 0"
TAG=$T LINES="vit:$B --mode vit;chr100:$B --workload chr100 --steps 3 --project-shards 8;lb:$B --block-len 100000 --steps 5;post77:$B --mode posterior --n-int 7 --steps 5;fv77:$B --n-int 7;vit77:$B --n-int 7 --mode vit;post55:$B --mode posterior --n-int 5 --steps 5;opt55:$B --mode optimize --steps 10 --warmup 3;fvint:$B --model introgression;rccl1:$B --dist 1 --backend nccl;n27fv:$B --n-int 3;n27vit:$B --n-int 3 --mode vit;n27post:$B --n-int 3 --mode posterior --steps 5" bash scripts/gpu_lines.sh
