# Sweep tests (every state count incl. 96/133/150) and the N > 72 bench lines after the
# configuration change.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_sweeps.py -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_sweeps.log 2>&1 || { tail -30 gpurun_out/pytest_sweeps.log; exit 1; }
tail -1 gpurun_out/pytest_sweeps.log
timeout -k 10 300 python bench.py --mode posterior --n-int 7 > gpurun_out/bench_post_7_7.json 2> gpurun_out/bench_post.err || { tail -5 gpurun_out/bench_post.err; exit 1; }
python scripts/bench_line.py gpurun_out/bench_post_7_7.json posterior77
timeout -k 10 300 python bench.py --mode fv --n-int 7 --check > gpurun_out/bench_fv_7_7.json 2> gpurun_out/bench_fv7.err || { tail -5 gpurun_out/bench_fv7.err; exit 1; }
python scripts/bench_line.py gpurun_out/bench_fv_7_7.json fv77
timeout -k 10 300 python bench.py --model introgression --mode fv --n-int 5 --check > gpurun_out/bench_intro_fv_5.json 2> gpurun_out/bench_ifv5.err || { tail -5 gpurun_out/bench_ifv5.err; exit 1; }
python scripts/bench_line.py gpurun_out/bench_intro_fv_5.json intro_fv55
