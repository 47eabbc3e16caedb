# the split last tile at N = 133: sweep tests, full-size (7,7) tests, posterior / forward lines
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r5q}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_sweeps.py -x -q -m gpu --timeout 120 --timeout-method thread > $O/pytest_sweeps.log 2>&1 || { tail -40 $O/pytest_sweeps.log; exit 1; }
tail -1 $O/pytest_sweeps.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_fullsize.py -x -q -m gpu -k "77 or 133" --timeout 300 --timeout-method thread > $O/pytest_full.log 2>&1 || { tail -40 $O/pytest_full.log; exit 1; }
tail -1 $O/pytest_full.log
B="--cpu-1core-cols 0 --host-path 0"
timeout -k 10 400 python bench.py $B --mode posterior --n-int 7 --steps 5 > $O/post77.json 2> $O/post77.err || { tail $O/post77.err; exit 1; }
python scripts/bench_line.py $O/post77.json post77
timeout -k 10 300 python bench.py $B --n-int 7 --steps 5 > $O/fv77.json 2> $O/fv77.err || { tail $O/fv77.err; exit 1; }
python scripts/bench_line.py $O/fv77.json fv77
echo done
