# Round 4: bulk Viterbi blocks traced by their own wave right after the sweep (product) vs the
# separate traceback after the join (previous tree's library, libitrails_hip_prev.so):
# sweep + full-size GPU tests, chr10 forward+Viterbi and Viterbi-only lines, kernel trace
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r4it}
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_sweeps.py tests/test_gpu_fullsize.py -x -q -m gpu --timeout 250 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
B="--cpu-1core-cols 0 --host-path 0"
for V in "" prev; do
  L=""; [ -n "$V" ] && L=itrails_amd/libitrails_hip_$V.so
  ITR_LIB=$L timeout -k 10 300 python bench.py $B > $O/fv$V.json 2> $O/fv$V.err || { tail $O/fv$V.err; exit 1; }
  python scripts/bench_line.py $O/fv$V.json "chr10 ${V:-intrace}"
  ITR_LIB=$L timeout -k 10 300 python bench.py $B --mode vit > $O/vit$V.json 2> $O/vit$V.err || { tail $O/vit$V.err; exit 1; }
  python scripts/bench_line.py $O/vit$V.json "vit ${V:-intrace}"
done
P="python3 bench.py --steps 3 --warmup 1 --verify 0 $B"
timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d $O/prof -o trace --output-format csv -- $P > $O/prof_trace.log 2>&1 || { tail $O/prof_trace.log; exit 1; }
find $O/prof -name "*kernel_stats.csv" -exec head -9 {} \;
echo done
