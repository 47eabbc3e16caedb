# Round 3: matrix-core chain with four accumulators per group: posterior parity + (7,7) bench
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r3pa
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_sweeps.py tests/test_gpu_fullsize.py -x -q -m gpu --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
B="--cpu-1core-cols 0 --host-path 0"
timeout -k 10 300 python bench.py $B --mode posterior --n-int 7 --steps 5 > $O/post77.json 2> $O/post77.err || { tail $O/post77.err; exit 1; }
python scripts/bench_line.py $O/post77.json post77
timeout -k 10 300 python bench.py $B --mode posterior --n-int 7 --steps 5 --verify 0 > $O/post77b.json 2> $O/post77b.err || { tail $O/post77b.err; exit 1; }
python scripts/bench_line.py $O/post77b.json post77_2
timeout -k 10 300 python bench.py $B --verify 0 > $O/fv.json 2> $O/fv.err || { tail $O/fv.err; exit 1; }
python scripts/bench_line.py $O/fv.json chr10
