cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_dense.py tests/test_gpu_model.py tests/test_gpu_distributed.py tests/test_cli.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_pref.log 2>&1 || { tail -30 gpurun_out/pytest_pref.log; exit 1; }
tail -1 gpurun_out/pytest_pref.log
timeout -k 10 300 python -u scripts/prof_build.py 5 3 > gpurun_out/prof_build.log 2>&1 || { tail -5 gpurun_out/prof_build.log; exit 1; }
grep -E "first|warm|enqueue" gpurun_out/prof_build.log
timeout -k 10 300 python bench.py --mode optimize --steps 10 --warmup 2 --verify 0 --host-path 0 --cpu-1core-cols 0 > gpurun_out/bench_opt.json 2> gpurun_out/bench_opt.err || { tail -5 gpurun_out/bench_opt.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/bench_opt.json')); print(d['value'], d['ms_per_step'], d.get('build_ms'))"
