# Round 3: posterior reductions (VALU + matrix-core backward) parity + bench; long-block fv
# timeline (few-blocks partition)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r3i
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_sweeps.py tests/test_gpu_fullsize.py -x -q -m gpu --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python bench.py --mode posterior --n-int 7 --cpu-1core-cols 0 --host-path 0 --steps 5 > $O/post77.json 2> $O/post77.err || { tail $O/post77.err; exit 1; }
python scripts/bench_line.py $O/post77.json post77
timeout -k 10 200 python bench.py --mode posterior --n-int 7 --block-len 20000 --mbp 0.02 --cpu-1core-cols 0 --host-path 0 --verify 0 --steps 3 > $O/post1.json 2> $O/post1.err || { tail $O/post1.err; exit 1; }
python scripts/bench_line.py $O/post1.json post_one_block_20000
timeout -k 10 300 python bench.py --mode posterior --cpu-1core-cols 0 --host-path 0 --steps 5 > $O/post55.json 2> $O/post55.err || { tail $O/post55.err; exit 1; }
python scripts/bench_line.py $O/post55.json post55
timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d $O/lb -o lb --output-format csv -- python3 bench.py --block-len 100000 --mbp 10 --cpu-1core-cols 0 --host-path 0 --verify 0 --steps 2 --warmup 1 > $O/lb.log 2>&1 || { tail $O/lb.log; exit 1; }
grep '^{' $O/lb.log > $O/lb.json && python scripts/bench_line.py $O/lb.json longblock_traced
