# Round 4: several long Viterbi blocks per reserved CU at a time (kLongPerCu: the planner
# divides the long set's CU bins by it; experiment library ITR_LONG_PER_CU): chr10
# forward+Viterbi (20 steps, twice), Viterbi-only, chr100 N = 1 + world-8 shard projection
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r4lp}
mkdir -p $O
B="--cpu-1core-cols 0 --host-path 0 --verify 0"
show() { python3 -c "
import json; d=json.loads(open('$1').read().strip().splitlines()[-1]); s=d.get('shard_projection',{})
print('$2', 'N1', d['ms_per_step'], 'shards', s.get('per_shard_ms'), 'max', s.get('max_ms'), 'x', s.get('projected_speedup'))"; }
export ITR_LIB=itrails_amd/libitrails_hip_exp.so
for L in ${LPCS:-1 2 3}; do
  export ITR_LONG_PER_CU=$L
  for i in 1 2; do
    timeout -k 10 300 python bench.py $B --steps 20 --warmup 3 > $O/fv_$L.$i.json 2> $O/fv_$L.$i.err || { tail $O/fv_$L.$i.err; exit 1; }
    python scripts/bench_line.py $O/fv_$L.$i.json "chr10 long_per_cu $L run $i"
  done
  timeout -k 10 300 python bench.py $B --mode vit --steps 20 --warmup 3 > $O/vit_$L.json 2> $O/vit_$L.err || { tail $O/vit_$L.err; exit 1; }
  python scripts/bench_line.py $O/vit_$L.json "vit long_per_cu $L"
  timeout -k 10 400 python bench.py $B --workload chr100 --steps 5 --warmup 2 --project-shards 8 > $O/sh_$L.json 2> $O/sh_$L.err || { tail $O/sh_$L.err; exit 1; }
  show $O/sh_$L.json "chr100 long_per_cu $L"
done
echo done
