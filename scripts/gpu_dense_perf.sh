# Dense kernels: GPU tests of dense.hip and the model build, cold/warm build times, the
# optimize evaluation loop, and a batched-GEMM rate probe.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_dense.py tests/test_gpu_model.py -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_dense.log 2>&1 || { tail -30 gpurun_out/pytest_dense.log; exit 1; }
tail -1 gpurun_out/pytest_dense.log
timeout -k 10 300 python scripts/model_timing.py 3 5 7 > gpurun_out/model_timing.log 2>&1 || { tail -20 gpurun_out/model_timing.log; exit 1; }
grep cold gpurun_out/model_timing.log
timeout -k 10 300 python scripts/gemm_rate.py > gpurun_out/gemm_rate.log 2>&1 || { tail -20 gpurun_out/gemm_rate.log; exit 1; }
cat gpurun_out/gemm_rate.log
timeout -k 10 300 python bench.py --mode optimize --n-int 5 --steps 5 --warmup 1 > gpurun_out/bench_opt.json 2>/dev/null || exit 1
python -c "import json;d=json.load(open('gpurun_out/bench_opt.json'));print('optimize (5,5)', d['value'], 'eval/s build_ms', d['build_ms'])"
