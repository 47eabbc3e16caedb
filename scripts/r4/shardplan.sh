# Round 4: the makespan estimate after the per-block pruned step (experiment library):
# ITR_BULK_CU (bulk cost, product 180e-9) with ITR_PRUNE_COL scaled to keep the prune length,
# ITR_WAVE_LAT (the long-set threshold's per-wave step, product 800e-9); chr100 world-8
# shards (projection) and chr10 forward+Viterbi (20 steps)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r4sp}
mkdir -p $O
B="--cpu-1core-cols 0 --host-path 0 --verify 0"
show() { python3 -c "
import json; d=json.loads(open('$1').read().strip().splitlines()[-1]); s=d.get('shard_projection',{})
print('$2', 'N1', d['ms_per_step'], 'shards', s.get('per_shard_ms'), 'max', s.get('max_ms'), 'x', s.get('projected_speedup'))"; }
export ITR_LIB=itrails_amd/libitrails_hip_exp.so
for V in ${VARS:-180e-9:1.4e-6:800e-9 150e-9:1.17e-6:800e-9 130e-9:1.01e-6:800e-9 180e-9:1.4e-6:650e-9 150e-9:1.17e-6:650e-9}; do
  IFS=: read BU PC WL <<< "$V"
  export ITR_BULK_CU=$BU ITR_PRUNE_COL=$PC ITR_WAVE_LAT=$WL
  timeout -k 10 400 python bench.py $B --workload chr100 --steps 5 --warmup 2 --project-shards 8 > $O/sh_$V.json 2> $O/sh_$V.err || { tail $O/sh_$V.err; exit 1; }
  show $O/sh_$V.json "chr100 bulk:pcol:wlat $V"
  timeout -k 10 300 python bench.py $B --steps 20 --warmup 3 > $O/fv_$V.json 2> $O/fv_$V.err || { tail $O/fv_$V.err; exit 1; }
  python scripts/bench_line.py $O/fv_$V.json "chr10 bulk:pcol:wlat $V"
done
echo done
