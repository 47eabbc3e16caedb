cd $GRAFT_REPO_ROOT
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || exit 1
python -c "from itrails_amd.build import build; build(force=True, diag=True)" >> gpurun_out/build.log 2>&1 || exit 1
timeout -k 10 600 python -m pytest tests -x -q -m gpu --timeout=300 --timeout-method=thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python scripts/diag_probe.py 2>&1 | tee gpurun_out/diag.log
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --cpu-sample 0 > gpurun_out/bench1.json 2> gpurun_out/bench1.err; rc=$?
cat gpurun_out/bench1.json
