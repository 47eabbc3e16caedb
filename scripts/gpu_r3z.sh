# Round 3: one partition per thread; standalone Viterbi on the same reserved sets; long blocks
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r3z
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_sweeps.py tests/test_gpu_fullsize.py tests/test_gpu_distributed.py -x -q -m gpu --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
B="--cpu-1core-cols 0 --host-path 0"
timeout -k 10 300 python bench.py $B > $O/fv.json 2> $O/fv.err || { tail $O/fv.err; exit 1; }
python scripts/bench_line.py $O/fv.json chr10
timeout -k 10 300 python bench.py $B --block-len 100000 --steps 5 > $O/lb.json 2> $O/lb.err || { tail $O/lb.err; exit 1; }
python scripts/bench_line.py $O/lb.json longblock
timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d $O/lbp -o lb --output-format csv -- python3 scripts/kernel_lab.py --block-len 100000 --which fv --reps 2 > $O/lbp.log 2>&1 || { tail $O/lbp.log; exit 1; }
echo traced
