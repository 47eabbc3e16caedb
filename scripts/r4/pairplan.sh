# Round 4: pairing long blocks on the reserved CUs by the planner (kVitPair: the paired step
# time; pairs only when the longest block fits the makespan at it), experiment library:
# ITR_VIT_PAIR values and the unpaired plan (ITR_LONG_PER_CU=1); chr10 forward+Viterbi (20
# steps, twice), Viterbi-only, chr100 N = 1 + world-8 shard projection
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r4pp}
mkdir -p $O
B="--cpu-1core-cols 0 --host-path 0 --verify 0"
show() { python3 -c "
import json; d=json.loads(open('$1').read().strip().splitlines()[-1]); s=d.get('shard_projection',{})
print('$2', 'N1', d['ms_per_step'], 'shards', s.get('per_shard_ms'), 'max', s.get('max_ms'), 'x', s.get('projected_speedup'))"; }
export ITR_LIB=itrails_amd/libitrails_hip_exp.so
for V in ${VARS:-unpaired 360e-9 400e-9 330e-9}; do
  unset ITR_LONG_PER_CU ITR_VIT_PAIR
  if [ $V = unpaired ]; then export ITR_LONG_PER_CU=1; else export ITR_VIT_PAIR=$V; fi
  for i in 1 2; do
    timeout -k 10 300 python bench.py $B --steps 20 --warmup 3 > $O/fv_$V.$i.json 2> $O/fv_$V.$i.err || { tail $O/fv_$V.$i.err; exit 1; }
    python scripts/bench_line.py $O/fv_$V.$i.json "chr10 pair $V run $i"
  done
  timeout -k 10 300 python bench.py $B --mode vit --steps 20 --warmup 3 > $O/vit_$V.json 2> $O/vit_$V.err || { tail $O/vit_$V.err; exit 1; }
  python scripts/bench_line.py $O/vit_$V.json "vit pair $V"
  timeout -k 10 400 python bench.py $B --workload chr100 --steps 5 --warmup 2 --project-shards 8 > $O/sh_$V.json 2> $O/sh_$V.err || { tail $O/sh_$V.err; exit 1; }
  show $O/sh_$V.json "chr100 pair $V"
done
echo done
