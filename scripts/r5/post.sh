# (7,7) posterior A/B: parity tests touching the matrix-core posterior, then the post77 line
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r5post}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu -k "post or 133 or 77" --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
B="--cpu-1core-cols 0 --host-path 0"
timeout -k 10 400 python bench.py $B --mode posterior --n-int 7 --steps 5 > $O/post77.json 2> $O/post77.err || { tail $O/post77.err; exit 1; }
python scripts/bench_line.py $O/post77.json post77
timeout -s KILL 200 rocprofv3 --kernel-trace --stats -d $O/prof -o trace --output-format csv -- python3 bench.py $B --mode posterior --n-int 7 --steps 2 --warmup 1 --verify 0 > $O/prof.log 2>&1 || { tail $O/prof.log; exit 1; }
python - $O/prof/trace_kernel_stats.csv <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if float(r["TotalDurationNs"]) > 1e6: print(r["Name"][:90], r["Calls"], round(float(r["AverageNs"])/1e6, 3), "ms")
PY
echo done
