# Round 4: bound-pruned per-wave Viterbi iteration: sweep GPU tests, vit / fv bench lines,
# kernel trace of the vit bench
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r4q}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_sweeps.py -x -q -m gpu --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
B="--cpu-1core-cols 0 --host-path 0"
timeout -k 10 300 python bench.py $B --mode vit > $O/vit.json 2> $O/vit.err || { tail $O/vit.err; exit 1; }
python scripts/bench_line.py $O/vit.json vit
timeout -k 10 300 python bench.py $B > $O/fv.json 2> $O/fv.err || { tail $O/fv.err; exit 1; }
python scripts/bench_line.py $O/fv.json chr10
P="python3 bench.py --steps 3 --warmup 1 --verify 0 --mode vit $B"
timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d $O/prof -o trace --output-format csv -- $P > $O/prof_trace.log 2>&1 || { tail $O/prof_trace.log; exit 1; }
find $O/prof -name "*kernel_stats.csv" -exec head -12 {} \;
echo done
