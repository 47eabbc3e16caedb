# GPU box: default bench vs --concurrent 1, alternating, CPU baseline and host leg skipped.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for i in 1 2 3; do
  for c in 0 1; do
    timeout -k 10 120 python bench.py --cpu-sample 0 --host-path 0 --steps 10 --concurrent $c > gpurun_out/concab_${c}_${i}.json 2>/dev/null || exit 1
    python -c "import json,sys; d=json.load(open('gpurun_out/concab_${c}_${i}.json')); print('concurrent=$c', d['value'], d['ms_per_step'])"
  done
done
