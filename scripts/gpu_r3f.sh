# Round 3: sweep parity (posterior global normalisation, new long set), then benches:
# fv (default, twice), posterior (7,7), optimize (5,5)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${TAG:-r3f}
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_sweeps.py tests/test_gpu_fullsize.py -x -q -m gpu --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for i in 1 2; do
timeout -k 10 300 python bench.py --verify 0 --cpu-1core-cols 0 --host-path 0 --steps 10 > $O/bench$i.json 2> $O/bench$i.err || { tail $O/bench$i.err; exit 1; }
python scripts/bench_line.py $O/bench$i.json fv$i
done
timeout -k 10 300 python bench.py --mode posterior --n-int 7 --cpu-1core-cols 0 --host-path 0 --steps 5 > $O/post77.json 2> $O/post77.err || { tail $O/post77.err; exit 1; }
python scripts/bench_line.py $O/post77.json post77
timeout -k 10 300 python bench.py --mode optimize --cpu-1core-cols 0 --host-path 0 --steps 10 > $O/opt55.json 2> $O/opt55.err || { tail $O/opt55.err; exit 1; }
python scripts/bench_line.py $O/opt55.json opt55
