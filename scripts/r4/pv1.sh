# Round 4: first GPU run of the prediction-and-verification Viterbi: sweep tests, full-size
# tests, chr10 and long-block benches
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r4b}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_sweeps.py -x -q -m gpu --timeout 120 --timeout-method thread > $O/pytest_sweeps.log 2>&1 || { tail -40 $O/pytest_sweeps.log; exit 1; }
tail -1 $O/pytest_sweeps.log
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
B="--cpu-1core-cols 0 --host-path 0"
timeout -k 10 300 python bench.py $B > $O/bench_fv.json 2> $O/bench_fv.err || { tail $O/bench_fv.err; exit 1; }
python scripts/bench_line.py $O/bench_fv.json chr10
timeout -k 10 300 python bench.py $B --block-len 100000 --steps 5 > $O/lb.json 2> $O/lb.err || { tail $O/lb.err; exit 1; }
python scripts/bench_line.py $O/lb.json longblock
echo done
