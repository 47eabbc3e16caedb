# Introgression model: GPU parity tests against the reference's goldens, then bench lines
# (forward+Viterbi on the device-built (3,3) and (5,5) int models, int-optimize loop).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_model.py tests/test_cli_int.py -x -q -m gpu -k "introgression or int_" --timeout 300 --timeout-method thread -s > gpurun_out/pytest_intro.log 2>&1 || { tail -30 gpurun_out/pytest_intro.log; exit 1; }
grep -E "built in|passed|failed" gpurun_out/pytest_intro.log
for cfg in "fv 3" "fv 5" "optimize 3" "optimize 5"; do
  set -- $cfg
  timeout -k 10 300 python bench.py --model introgression --mode $1 --n-int $2 --steps 5 --warmup 1 --check > gpurun_out/bench_intro_$1_$2.json 2> gpurun_out/bench_intro_$1_$2.err || { tail -5 gpurun_out/bench_intro_$1_$2.err; exit 1; }
  cat gpurun_out/bench_intro_$1_$2.json
done
