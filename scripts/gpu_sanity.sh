# GPU box: quick sanity of the built tree: sweep parity tests, smoke, default bench.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_sweeps.py tests/test_gpu_fullsize.py tests/test_gpu_distributed.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/pytest_sanity.log 2>&1 || { tail -30 gpurun_out/pytest_sanity.log; exit 1; }
tail -1 gpurun_out/pytest_sanity.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tail -1
timeout -k 10 300 python bench.py > gpurun_out/bench_sanity.json 2> gpurun_out/bench_sanity.err || { tail gpurun_out/bench_sanity.err; exit 1; }
python scripts/bench_line.py gpurun_out/bench_sanity.json final
