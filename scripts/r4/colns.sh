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

unset ITR_LIB
timeout -k 10 300 python -u -m pytest tests/test_gpu_model.py -x -q -m gpu --timeout 200 --timeout-method thread > $O/pytest_model.log 2>&1 || { tail -30 $O/pytest_model.log; exit 1; }
tail -1 $O/pytest_model.log
timeout -k 10 300 python bench.py --cpu-1core-cols 0 --host-path 0 --mode optimize > $O/opt.json 2> $O/opt.err || { tail $O/opt.err; exit 1; }
python scripts/bench_line.py $O/opt.json optimize
timeout -k 10 200 python3 scripts/prof_build.py 5 8 > $O/prof_build.log 2>&1 || { tail $O/prof_build.log; exit 1; }
head -3 $O/prof_build.log
echo done
