# GPU box: partition rule on chr100 / chr10 / long blocks; sweep parity tests first.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_sweeps.py tests/test_gpu_fullsize.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_final.log 2>&1 || { tail -30 gpurun_out/pytest_final.log; exit 1; }
tail -1 gpurun_out/pytest_final.log
timeout -k 10 400 python bench.py --workload chr100 --steps 3 --warmup 1 --cpu-1core-cols 0 --host-path 0 > gpurun_out/m_chr100b.json 2> gpurun_out/m.err || { tail gpurun_out/m.err; exit 1; }
python scripts/bench_line.py gpurun_out/m_chr100b.json chr100
timeout -k 10 200 python bench.py --cpu-1core-cols 0 --host-path 0 > gpurun_out/m_chr10b.json 2> gpurun_out/m.err || { tail gpurun_out/m.err; exit 1; }
python scripts/bench_line.py gpurun_out/m_chr10b.json chr10
timeout -k 10 300 python bench.py --block-len 100000 --steps 3 --warmup 1 --cpu-1core-cols 0 --host-path 0 > gpurun_out/m_lb.json 2> gpurun_out/m.err || { tail gpurun_out/m.err; exit 1; }
python scripts/bench_line.py gpurun_out/m_lb.json longblock
