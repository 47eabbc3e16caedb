# GPU box: one-block-per-wave Viterbi: sweep + full-size parity tests, then the default bench.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_sweeps.py tests/test_gpu_fullsize.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_wave.log 2>&1 || { tail -40 gpurun_out/pytest_wave.log; exit 1; }
tail -2 gpurun_out/pytest_wave.log
timeout -k 10 400 python bench.py --cpu-1core-cols 0 --host-path 0 > gpurun_out/bench_wave.json 2> gpurun_out/bench_wave.err || { tail gpurun_out/bench_wave.err; exit 1; }
python scripts/bench_line.py gpurun_out/bench_wave.json wave
