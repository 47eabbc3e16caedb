# Round 4: kMixGroupCol calibration after the mixed launch serves a forward without VALU
# tasks (experiment library, ITR_URGENT_COLNS): chr100 N = 1 + 8-shard projection, chr10
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r4y}
mkdir -p $O
B="--cpu-1core-cols 0 --host-path 0 --verify 0"
show() { python3 -c "
import json; d=json.loads(open('$1').read().strip().splitlines()[-1]); s=d.get('shard_projection',{})
print('$2', 'N1', d['ms_per_step'], 'shards', s.get('per_shard_ms'), 'max', s.get('max_ms'), 'x', s.get('projected_speedup'))"; }
export ITR_LIB=itrails_amd/libitrails_hip_exp.so
for C in ${COLNS:-500 800 1100 1400 2000}; do
  ITR_URGENT_COLNS=$C timeout -k 10 400 python bench.py $B --workload chr100 --steps 5 --warmup 2 --project-shards 8 > $O/sh_c$C.json 2> $O/sh_c$C.err || { tail $O/sh_c$C.err; exit 1; }
  show $O/sh_c$C.json "colns $C"
  ITR_URGENT_COLNS=$C timeout -k 10 300 python bench.py $B > $O/fv_c$C.json 2> $O/fv_c$C.err || { tail $O/fv_c$C.err; exit 1; }
  python scripts/bench_line.py $O/fv_c$C.json "chr10 colns $C"
done
echo done
