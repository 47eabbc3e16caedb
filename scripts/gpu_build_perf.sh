# Model-build throughput: GPU parity of every model golden, cold/warm device build times,
# and the itrails-optimize / itrails-int-optimize evaluation loops (BASELINE config 5).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_model.py -q -m gpu --timeout 300 --timeout-method thread -s > gpurun_out/pytest_model.log 2>&1 || { tail -30 gpurun_out/pytest_model.log; exit 1; }
grep -E "built in|passed|failed" gpurun_out/pytest_model.log
timeout -k 10 300 python scripts/model_timing.py 3 5 7 > gpurun_out/model_timing.log 2>&1 || { tail -20 gpurun_out/model_timing.log; exit 1; }
grep -E "cold" gpurun_out/model_timing.log
for m in itrails introgression; do
  timeout -k 10 300 python bench.py --model $m --mode optimize --n-int 5 --steps 5 --warmup 1 > gpurun_out/bench_opt_$m.json 2> gpurun_out/bench_opt_$m.err || { tail -5 gpurun_out/bench_opt_$m.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/bench_opt_$m.json'));print('$m', d['value'], d['unit'], 'build_ms', d.get('build_ms'), 'fwd', d['roofline']['forward_ms'])"
done
