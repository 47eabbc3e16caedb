cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_distributed.py tests/test_gpu_model.py -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_split.log 2>&1 || { tail -40 gpurun_out/pytest_split.log; exit 1; }
grep -E "PASS|FAIL|passed|failed" gpurun_out/pytest_split.log | tail -8
