# Round 3 kernel lab 3: the mixed per-wave launch in the combined call; parity first.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/lab3
L=gpurun_out/lab3/lab.txt
: > $L
timeout -k 10 300 python -u -m pytest tests/test_gpu_sweeps.py tests/test_gpu_fullsize.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/lab3/pytest.log 2>&1 || { tail -30 gpurun_out/lab3/pytest.log; exit 1; }
tail -1 gpurun_out/lab3/pytest.log
run() { timeout -k 10 120 env "$@" >> $L 2>&1 || { tail $L; exit 1; }; }
run python scripts/kernel_lab.py --mean-block 2000 --which fwd,vit,fv --tag chr10 --check 1
run python scripts/kernel_lab.py --mean-block 250 --which vit,fv --tag short
run python scripts/kernel_lab.py --block-len 100000 --which fv --tag longblock
cat $L
for i in 1 2; do
timeout -k 10 300 python bench.py --verify 0 --cpu-1core-cols 0 --host-path 0 --steps 10 > gpurun_out/lab3/bench$i.json 2> gpurun_out/lab3/bench$i.err || { tail gpurun_out/lab3/bench$i.err; exit 1; }
python scripts/bench_line.py gpurun_out/lab3/bench$i.json run$i
done
