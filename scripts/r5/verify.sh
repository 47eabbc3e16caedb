# every GPU test, smoke, then the default bench and the (7,7) posterior line
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r5v}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
B="--cpu-1core-cols 0 --host-path 0"
timeout -k 10 400 python bench.py $B > $O/bench_fv.json 2> $O/bench_fv.err || { tail $O/bench_fv.err; exit 1; }
python scripts/bench_line.py $O/bench_fv.json chr10
timeout -k 10 400 python bench.py $B --mode posterior --n-int 7 --steps 5 > $O/post77.json 2> $O/post77.err || { tail $O/post77.err; exit 1; }
python scripts/bench_line.py $O/post77.json post77

timeout -k 10 400 python bench.py $B --mode posterior --n-int 5 --steps 5 > $O/post55.json 2> $O/post55.err || { tail $O/post55.err; exit 1; }
python scripts/bench_line.py $O/post55.json post55
echo done
