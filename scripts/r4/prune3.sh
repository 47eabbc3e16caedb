# Round 4: pruned per-wave Viterbi: product (rolled tile loop) vs unrolled-tile variant
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r4s}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_sweeps.py tests/test_gpu_rows.py tests/test_gpu_dense.py tests/test_gpu_model.py -x -q -m gpu --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
B="--cpu-1core-cols 0 --host-path 0"
for V in "" unroll; do
  L=""; [ -n "$V" ] && L="itrails_amd/libitrails_hip_$V.so"
  ITR_LIB=$L timeout -k 10 300 python bench.py $B --mode vit > $O/vit$V.json 2> $O/vit$V.err || { tail $O/vit$V.err; exit 1; }
  python scripts/bench_line.py $O/vit$V.json "vit $V"
  ITR_LIB=$L timeout -k 10 300 python bench.py $B > $O/fv$V.json 2> $O/fv$V.err || { tail $O/fv$V.err; exit 1; }
  python scripts/bench_line.py $O/fv$V.json "chr10 $V"
done
P="python3 bench.py --steps 3 --warmup 1 --verify 0 --mode vit $B"
timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d $O/prof -o trace --output-format csv -- $P > $O/prof_trace.log 2>&1 || { tail $O/prof_trace.log; exit 1; }
find $O/prof -name "*kernel_stats.csv" -exec head -4 {} \;
echo done
