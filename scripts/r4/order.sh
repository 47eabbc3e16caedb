# Round 4: the forward+Viterbi call with the bulk launch enqueued first and one counter memset
# (the step's critical path starts ~10 API calls earlier): sweep and full-size tests, then
# chr10 forward+Viterbi (20 steps, three runs), Viterbi-only and chr100
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r4or}
mkdir -p $O
B="--cpu-1core-cols 0 --host-path 0 --verify 0"
timeout -k 10 600 python -u -m pytest tests/test_gpu_sweeps.py tests/test_gpu_fullsize.py -x -q -m gpu --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for i in 1 2 3; do
  timeout -k 10 300 python bench.py $B --steps 20 --warmup 3 > $O/fv.$i.json 2> $O/fv.$i.err || { tail $O/fv.$i.err; exit 1; }
  python scripts/bench_line.py $O/fv.$i.json "chr10 run $i"
done
timeout -k 10 300 python bench.py $B --mode vit --steps 20 --warmup 3 > $O/vit.json 2> $O/vit.err || { tail $O/vit.err; exit 1; }
python scripts/bench_line.py $O/vit.json "vit"
timeout -k 10 300 python bench.py $B --workload chr100 --steps 3 --warmup 1 > $O/c100.json 2> $O/c100.err || { tail $O/c100.err; exit 1; }
python scripts/bench_line.py $O/c100.json "chr100"
echo done
