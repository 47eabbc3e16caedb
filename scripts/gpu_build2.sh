# model build rewrite: dense + model GPU tests, build profile
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_dense.py tests/test_gpu_model.py -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_build2.log 2>&1 || { tail -40 gpurun_out/pytest_build2.log; exit 1; }
grep -E "passed|failed" gpurun_out/pytest_build2.log | tail -3
timeout -k 10 300 python -u scripts/prof_build.py 5 3 > gpurun_out/prof_build.log 2>&1 || { tail -20 gpurun_out/prof_build.log; exit 1; }
head -30 gpurun_out/prof_build.log
