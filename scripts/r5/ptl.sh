# kernel trace of the (7,7) posterior (product library) -> timeline of its last call
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r5ptl}
mkdir -p $O
timeout -s KILL 200 rocprofv3 --kernel-trace --stats -d $O/prof -o trace --output-format csv -- python3 bench.py --cpu-1core-cols 0 --host-path 0 --verify 0 --mode posterior --n-int 7 --steps 2 --warmup 1 > $O/prof.log 2>&1 || { tail $O/prof.log; exit 1; }
python scripts/r5/ptimeline.py $O/prof/trace_kernel_trace.csv
