# Round 3: long blocks' traceback on their reserved CUs: parity + chr10 bench (x2) + chr100
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r3tb
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_sweeps.py tests/test_gpu_fullsize.py tests/test_gpu_distributed.py -x -q -m gpu --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
B="--cpu-1core-cols 0 --host-path 0"
timeout -k 10 300 python bench.py $B > $O/fv.json 2> $O/fv.err || { tail $O/fv.err; exit 1; }
python scripts/bench_line.py $O/fv.json chr10
timeout -k 10 300 python bench.py $B --verify 0 > $O/fv2.json 2> $O/fv2.err || { tail $O/fv2.err; exit 1; }
python scripts/bench_line.py $O/fv2.json chr10_2
timeout -k 10 300 python bench.py $B --workload chr100 --steps 3 > $O/chr100.json 2> $O/chr100.err || { tail $O/chr100.err; exit 1; }
python scripts/bench_line.py $O/chr100.json chr100
