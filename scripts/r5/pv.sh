# pruned Viterbi at N = 95 / 133: sweep tests, full-size tests, benches (fv77, intro95, vit)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r5g}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_sweeps.py -x -v -m gpu --timeout 120 --timeout-method thread > $O/pytest_sweeps.log 2>&1 || { tail -40 $O/pytest_sweeps.log; exit 1; }
tail -1 $O/pytest_sweeps.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_fullsize.py -x -v -m gpu -k "77 or intro95" --timeout 300 --timeout-method thread > $O/pytest_full.log 2>&1 || { tail -40 $O/pytest_full.log; exit 1; }
tail -1 $O/pytest_full.log
B="--cpu-1core-cols 0 --host-path 0"
timeout -k 10 300 python bench.py $B --n-int 7 > $O/fv77.json 2> $O/fv77.err || { tail $O/fv77.err; exit 1; }
python scripts/bench_line.py $O/fv77.json fv77
timeout -k 10 300 python bench.py $B --n-int 7 --mode vit > $O/vit77.json 2> $O/vit77.err || { tail $O/vit77.err; exit 1; }
python scripts/bench_line.py $O/vit77.json vit77
timeout -k 10 300 python bench.py $B --model introgression > $O/fvint.json 2> $O/fvint.err || { tail $O/fvint.err; exit 1; }
python scripts/bench_line.py $O/fvint.json fv_intro95
timeout -k 10 300 python bench.py $B --model introgression --mode vit > $O/vitint.json 2> $O/vitint.err || { tail $O/vitint.err; exit 1; }
python scripts/bench_line.py $O/vitint.json vit_intro95
timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d $O/prof -o trace --output-format csv -- python3 bench.py $B --n-int 7 --mode vit --steps 3 --warmup 1 --verify 0 > $O/prof.log 2>&1 || { tail $O/prof.log; exit 1; }
head -8 $O/prof/trace_kernel_stats.csv | cut -c1-150
echo done
