# Round 3: kernel trace of the planned forward+Viterbi call (chr10, chr100) for the timeline
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r3w
mkdir -p $O
timeout -s KILL 200 rocprofv3 --kernel-trace --stats -d $O/prof -o fv --output-format csv -- python3 scripts/prof_sweeps.py 4 fv > $O/trace.log 2>&1 || { tail $O/trace.log; exit 1; }
echo traced
