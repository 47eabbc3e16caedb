# Round 3: reserved CUs steal from the mixed queue; forward staging lane constants.  Parity,
# chr10 bench, chr100 at N=1, posterior (7,7), optimize (5,5), long blocks
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r3o}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_sweeps.py tests/test_gpu_fullsize.py -x -q -m gpu --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
B="--cpu-1core-cols 0 --host-path 0"
timeout -k 10 200 python bench.py $B > $O/fv.json 2> $O/fv.err || { tail $O/fv.err; exit 1; }
python scripts/bench_line.py $O/fv.json chr10
timeout -k 10 300 python bench.py $B --workload chr100 --verify 0 --steps 3 > $O/chr100.json 2> $O/chr100.err || { tail $O/chr100.err; exit 1; }
python scripts/bench_line.py $O/chr100.json chr100
timeout -k 10 300 python bench.py $B --mode posterior --n-int 7 --steps 5 > $O/post77.json 2> $O/post77.err || { tail $O/post77.err; exit 1; }
python scripts/bench_line.py $O/post77.json post77
timeout -k 10 300 python bench.py $B --mode optimize --steps 10 --warmup 3 > $O/opt55.json 2> $O/opt55.err || { tail $O/opt55.err; exit 1; }
python scripts/bench_line.py $O/opt55.json opt55
timeout -k 10 300 python bench.py $B --block-len 100000 --steps 3 > $O/lb.json 2> $O/lb.err || { tail $O/lb.err; exit 1; }
python scripts/bench_line.py $O/lb.json longblock
