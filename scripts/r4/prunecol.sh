# Round 4: calibration of kPruneCol (capi.cpp): a per-wave Viterbi block takes the
# bound-pruned step when its length x kPruneCol fits within the plan's expected makespan.
# chr10 forward+Viterbi and Viterbi-only (20 steps each), chr100 N = 1 + world-8 shard
# projection; off = every block on the full scan (experiment library).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r4pc}
mkdir -p $O
B="--cpu-1core-cols 0 --host-path 0 --verify 0"
show() { python3 -c "
import json; d=json.loads(open('$1').read().strip().splitlines()[-1]); s=d.get('shard_projection',{})
print('$2', 'N1', d['ms_per_step'], 'shards', s.get('per_shard_ms'), 'max', s.get('max_ms'), 'x', s.get('projected_speedup'))"; }
export ITR_LIB=itrails_amd/libitrails_hip_exp.so
for C in ${COLS:-off 2.0e-6 2.9e-6 4.0e-6 6.0e-6}; do
  if [ $C = off ]; then export ITR_PRUNE_LEN=0; unset ITR_PRUNE_COL; else unset ITR_PRUNE_LEN; export ITR_PRUNE_COL=$C; fi
  timeout -k 10 300 python bench.py $B --steps 20 --warmup 3 > $O/fv_$C.json 2> $O/fv_$C.err || { tail $O/fv_$C.err; exit 1; }
  python scripts/bench_line.py $O/fv_$C.json "chr10 col $C"
  timeout -k 10 300 python bench.py $B --mode vit --steps 20 --warmup 3 > $O/vit_$C.json 2> $O/vit_$C.err || { tail $O/vit_$C.err; exit 1; }
  python scripts/bench_line.py $O/vit_$C.json "vit col $C"
  timeout -k 10 400 python bench.py $B --workload chr100 --steps 5 --warmup 2 --project-shards 8 > $O/sh_$C.json 2> $O/sh_$C.err || { tail $O/sh_$C.err; exit 1; }
  show $O/sh_$C.json "chr100 col $C"
done
echo done
