# round 2, first measurement pass: VALU peak micro, all GPU tests, default bench (config 2),
# config 4 workload on one GPU (strong-scaling baseline)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 scripts/micro/valu_peak > gpurun_out/valu_peak.txt 2>&1 || { cat gpurun_out/valu_peak.txt; exit 1; }
cat gpurun_out/valu_peak.txt
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 400 --timeout-method thread > gpurun_out/pytest_r2a.log 2>&1 || { tail -40 gpurun_out/pytest_r2a.log; exit 1; }
tail -3 gpurun_out/pytest_r2a.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_fv_r2a.json 2> gpurun_out/bench_fv_r2a.err || { tail gpurun_out/bench_fv_r2a.err; exit 1; }
cat gpurun_out/bench_fv_r2a.json
timeout -k 10 600 python bench.py --workload chr100 --steps 5 --warmup 2 --host-path 0 > gpurun_out/bench_chr100_n1_r2a.json 2> gpurun_out/bench_chr100_n1_r2a.err || { tail gpurun_out/bench_chr100_n1_r2a.err; exit 1; }
cat gpurun_out/bench_chr100_n1_r2a.json
