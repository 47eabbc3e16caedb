# Round 4: makespan floor of the VALU-task threshold (product) vs the fraction rule alone
# (experiment library, ITR_URGENT_COLNS=0): GPU sweep/full-size tests, chr10, chr100 N = 1
# with the 8-shard projection, 100 x 100 kbp
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r4x}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_sweeps.py tests/test_gpu_fullsize.py -x -q -m gpu --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
B="--cpu-1core-cols 0 --host-path 0"
show() { python3 -c "
import json; d=json.loads(open('$1').read().strip().splitlines()[-1]); s=d.get('shard_projection',{})
print('$2', 'N1', d['ms_per_step'], 'vit_eq', d.get('viterbi_equal'), 'shards', s.get('per_shard_ms'), 'max', s.get('max_ms'), 'x', s.get('projected_speedup'))"; }
for V in new old; do
  if [ $V = old ]; then export ITR_LIB=itrails_amd/libitrails_hip_exp.so ITR_URGENT_COLNS=0; fi
  timeout -k 10 300 python bench.py $B > $O/fv_$V.json 2> $O/fv_$V.err || { tail $O/fv_$V.err; exit 1; }
  python scripts/bench_line.py $O/fv_$V.json "chr10 $V"
  timeout -k 10 400 python bench.py $B --workload chr100 --steps 5 --warmup 2 --project-shards 8 > $O/sh_$V.json 2> $O/sh_$V.err || { tail $O/sh_$V.err; exit 1; }
  show $O/sh_$V.json "chr100 $V"
  timeout -k 10 300 python bench.py $B --block-len 100000 --steps 5 > $O/lb_$V.json 2> $O/lb_$V.err || { tail $O/lb_$V.err; exit 1; }
  python scripts/bench_line.py $O/lb_$V.json "longblock $V"
done
echo done
