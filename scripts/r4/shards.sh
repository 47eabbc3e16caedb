# Round 4: chr100 per-shard projection (8 shards) with the product plan and with the
# makespan-based urgent threshold of the experiment library (ITR_URGENT_COLNS)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r4u}
mkdir -p $O
B="--cpu-1core-cols 0 --host-path 0 --workload chr100 --steps 5 --warmup 2 --verify 0 --project-shards 8"
show() { python3 -c "
import json,sys; d=json.loads(open('$1').read().strip().splitlines()[-1]); s=d.get('shard_projection',{})
print('$2', 'N1', d['ms_per_step'], 'shards', s.get('per_shard_ms'), 'max', s.get('max_ms'), 'x', s.get('projected_speedup'))"; }
timeout -k 10 400 python bench.py $B > $O/base.json 2> $O/base.err || { tail $O/base.err; exit 1; }
show $O/base.json base
for C in ${COLNS:-700 1000 1400}; do
  ITR_LIB=itrails_amd/libitrails_hip_exp.so ITR_URGENT_COLNS=$C timeout -k 10 400 python bench.py $B > $O/c$C.json 2> $O/c$C.err || { tail $O/c$C.err; exit 1; }
  show $O/c$C.json colns$C
done
echo done
