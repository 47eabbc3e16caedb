# matrix-core sweeps after the deeper A-operand prefetch: sweep tests, posterior / forward lines
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r5m}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_sweeps.py -x -q -m gpu --timeout 120 --timeout-method thread > $O/pytest_sweeps.log 2>&1 || { tail -40 $O/pytest_sweeps.log; exit 1; }
tail -1 $O/pytest_sweeps.log
B="--cpu-1core-cols 0 --host-path 0"
timeout -k 10 400 python bench.py $B --mode posterior --n-int 7 --steps 5 > $O/post77.json 2> $O/post77.err || { tail $O/post77.err; exit 1; }
python scripts/bench_line.py $O/post77.json post77
timeout -k 10 300 python bench.py $B --n-int 7 --overlap 0 --steps 5 > $O/fv77.json 2> $O/fv77.err || { tail $O/fv77.err; exit 1; }
python scripts/bench_line.py $O/fv77.json fv77
timeout -k 10 300 python bench.py $B --mode optimize --steps 10 --warmup 3 > $O/opt55.json 2> $O/opt55.err || { tail $O/opt55.err; exit 1; }
python scripts/bench_line.py $O/opt55.json opt55
timeout -k 10 300 python bench.py $B --overlap 0 --verify 0 > $O/fv_sep.json 2> $O/fv_sep.err || { tail $O/fv_sep.err; exit 1; }
python scripts/bench_line.py $O/fv_sep.json chr10_separate_calls
timeout -k 10 300 python bench.py $B --verify 0 > $O/fv.json 2> $O/fv.err || { tail $O/fv.err; exit 1; }
python scripts/bench_line.py $O/fv.json chr10
echo done
