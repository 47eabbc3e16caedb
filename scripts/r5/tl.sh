# kernel timeline (begin/end of every launch) of the default bench's timed call
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-tl}
mkdir -p $O
timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d $O/tl -o tl --output-format csv -- python3 bench.py --steps 3 --warmup 3 --verify 0 --cpu-1core-cols 0 --host-path 0 $BENCH_ARGS > $O/tl.log 2>&1 || { tail $O/tl.log; exit 1; }
tail -1 $O/tl.log
