# Round 3: stealing after all reserved work; chr10 bench; kernel trace of the long-block call
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r3p}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_sweeps.py tests/test_gpu_fullsize.py -x -q -m gpu --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
B="--cpu-1core-cols 0 --host-path 0"
timeout -k 10 200 python bench.py $B > $O/fv.json 2> $O/fv.err || { tail $O/fv.err; exit 1; }
python scripts/bench_line.py $O/fv.json chr10
timeout -k 10 200 python bench.py $B --verify 0 > $O/fv2.json 2> $O/fv2.err || { tail $O/fv2.err; exit 1; }
python scripts/bench_line.py $O/fv2.json chr10_rerun
timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d $O/lb -o lb --output-format csv -- python3 bench.py --block-len 100000 --mbp 10 $B --verify 0 --steps 2 --warmup 1 > $O/lb.log 2>&1 || { tail $O/lb.log; exit 1; }
grep '^{' $O/lb.log > $O/lb.json && python scripts/bench_line.py $O/lb.json longblock_traced
