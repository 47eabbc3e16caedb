# Round 4: kPruneCol calibration, second pass (chr10 forward+Viterbi twice per value, 20
# steps; with ITR_BULK_CU the bulk cost of the makespan estimate too) and the chr100 shards
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r4pc2}
mkdir -p $O
B="--cpu-1core-cols 0 --host-path 0 --verify 0"
show() { python3 -c "
import json; d=json.loads(open('$1').read().strip().splitlines()[-1]); s=d.get('shard_projection',{})
print('$2', 'N1', d['ms_per_step'], 'shards', s.get('per_shard_ms'), 'max', s.get('max_ms'), 'x', s.get('projected_speedup'))"; }
export ITR_LIB=itrails_amd/libitrails_hip_exp.so
for CB in 2.0e-6:180e-9 1.4e-6:180e-9 1.0e-6:180e-9 2.0e-6:160e-9 1.6e-6:150e-9 2.0e-6:180e-9; do
  export ITR_PRUNE_COL=${CB%%:*} ITR_BULK_CU=${CB##*:}
  for i in 1 2; do
    timeout -k 10 300 python bench.py $B --steps 20 --warmup 3 > $O/fv_$CB.$i.json 2> $O/fv_$CB.$i.err || { tail $O/fv_$CB.$i.err; exit 1; }
    python scripts/bench_line.py $O/fv_$CB.$i.json "chr10 col:bulk $CB run $i"
  done
done
for CB in 2.0e-6:180e-9 1.4e-6:180e-9; do
  export ITR_PRUNE_COL=${CB%%:*} ITR_BULK_CU=${CB##*:}
  timeout -k 10 400 python bench.py $B --workload chr100 --steps 5 --warmup 2 --project-shards 8 > $O/sh_$CB.json 2> $O/sh_$CB.err || { tail $O/sh_$CB.err; exit 1; }
  show $O/sh_$CB.json "chr100 col:bulk $CB"
done
echo done
