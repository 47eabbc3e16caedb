# CU census, Viterbi hybrid parity (experiment library) + variants, config-1 CLI test
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 60 scripts/micro/cu_key > gpurun_out/cu_key.log 2>&1 || { cat gpurun_out/cu_key.log; exit 1; }
cat gpurun_out/cu_key.log
timeout -k 10 300 python -u -m pytest tests/test_cli.py -x -q -m gpu -k config1 --timeout 240 --timeout-method thread > gpurun_out/pytest_cli1.log 2>&1 || { tail -30 gpurun_out/pytest_cli1.log; exit 1; }
tail -2 gpurun_out/pytest_cli1.log
timeout -k 10 300 python -u scripts/cli_e2e.py > gpurun_out/cli_e2e.log 2>&1 || { tail -30 gpurun_out/cli_e2e.log; exit 1; }
tail -15 gpurun_out/cli_e2e.log
export ITR_LIB=$PWD/itrails_amd/libitrails_hip_exp.so
ITR_VIT_HYBRID=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_sweeps.py tests/test_gpu_fullsize.py -x -q -m gpu -k "viterbi or Viterbi" --timeout 300 --timeout-method thread > gpurun_out/pytest_vith2.log 2>&1 || { tail -40 gpurun_out/pytest_vith2.log; exit 1; }
tail -2 gpurun_out/pytest_vith2.log
: > gpurun_out/vith2.log
run() {  # label, env...
  lab=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps 10 --warmup 3 --verify 1 --host-path 0 --cpu-1core-cols 0 > gpurun_out/b.json 2>> gpurun_out/vith2.err || { echo "bench FAIL $lab"; tail -5 gpurun_out/vith2.err; exit 1; }
  python -c "
import json; d=json.load(open('gpurun_out/b.json')); r=d['roofline']
print('$lab', 'vit_ms', r['viterbi_ms'], 'tb_ms', r['traceback_ms'], 'fwd_ms', r['forward_ms'], 'value', d['value'], d['viterbi_equal'])" >> gpurun_out/vith2.log
}
run valu_only ITR_X=0 || exit 1
for f in 0.25 0.4; do
  run "ql4_wait_$f" ITR_VIT_HYBRID=1 ITR_VIT_URGENT_FRAC=$f || exit 1
  run "ql4_exit_$f" ITR_VIT_HYBRID=1 ITR_VIT_EXIT=1 ITR_VIT_URGENT_FRAC=$f || exit 1
  run "ql4_nocu_$f" ITR_VIT_HYBRID=1 ITR_VIT_NOCU=1 ITR_VIT_URGENT_FRAC=$f || exit 1
  run "ql2_wait_$f" ITR_VIT_HYBRID=2 ITR_VIT_URGENT_FRAC=$f || exit 1
done
cat gpurun_out/vith2.log
timeout -k 10 300 python -u scripts/prof_build.py 5 4 > gpurun_out/prof_build.log 2>&1 || { tail -20 gpurun_out/prof_build.log; exit 1; }
head -5 gpurun_out/prof_build.log
