# Round 4: chr100 shard projection (product + makespan-based urgent threshold), the (7,7)
# forward+Viterbi line, config 5 (optimize) and a kernel trace of the (5,5) rebuild
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r4w}
mkdir -p $O
B="--cpu-1core-cols 0 --host-path 0"
timeout -k 10 300 python bench.py $B --mode optimize > $O/opt.json 2> $O/opt.err || { tail $O/opt.err; exit 1; }
python scripts/bench_line.py $O/opt.json optimize
timeout -k 10 200 python3 scripts/prof_build.py 5 8 > $O/prof_build.log 2>&1 || { tail $O/prof_build.log; exit 1; }
head -3 $O/prof_build.log
timeout -s KILL 200 rocprofv3 --kernel-trace --stats -d $O/prof_build -o build --output-format csv -- python3 scripts/prof_build.py 5 8 > $O/prof_build_trace.log 2>&1 || { tail $O/prof_build_trace.log; exit 1; }
timeout -k 10 300 python bench.py $B --n-int 7 --verify 1 > $O/fv77.json 2> $O/fv77.err || { tail $O/fv77.err; exit 1; }
python scripts/bench_line.py $O/fv77.json "fv (7,7)"
S="$B --workload chr100 --steps 5 --warmup 2 --verify 0 --project-shards 8"
show() { python3 -c "
import json; d=json.loads(open('$1').read().strip().splitlines()[-1]); s=d.get('shard_projection',{})
print('$2', 'N1', d['ms_per_step'], 'shards', s.get('per_shard_ms'), 'max', s.get('max_ms'), 'x', s.get('projected_speedup'))"; }
timeout -k 10 400 python bench.py $S > $O/sh_base.json 2> $O/sh_base.err || { tail $O/sh_base.err; exit 1; }
show $O/sh_base.json base
for C in 700 1000 1400; do
  ITR_LIB=itrails_amd/libitrails_hip_exp.so ITR_URGENT_COLNS=$C timeout -k 10 400 python bench.py $S > $O/sh_c$C.json 2> $O/sh_c$C.err || { tail $O/sh_c$C.err; exit 1; }
  show $O/sh_c$C.json colns$C
done
echo done
