# Round 4 baseline on this round's boxes: GPU tests, smoke, default bench, long blocks
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r4a}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
timeout -k 10 400 python bench.py > $O/bench_fv.json 2> $O/bench_fv.err || { tail $O/bench_fv.err; exit 1; }
python scripts/bench_line.py $O/bench_fv.json chr10
B="--cpu-1core-cols 0 --host-path 0"
timeout -k 10 300 python bench.py $B --block-len 100000 --steps 5 > $O/lb.json 2> $O/lb.err || { tail $O/lb.err; exit 1; }
python scripts/bench_line.py $O/lb.json longblock
echo done
