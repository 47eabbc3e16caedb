# GPU box: default bench line (now with the host-buffer drop-in leg) and the (7,7)
# posterior line; each step time-limited, stop at the first failure.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python bench.py > gpurun_out/bench_host_fv.json 2> gpurun_out/bench_host_fv.err || { tail gpurun_out/bench_host_fv.err; exit 1; }
cat gpurun_out/bench_host_fv.json
timeout -k 10 300 python bench.py --mode posterior --n-int 7 --cpu-sample 200000 > gpurun_out/bench_host_post7.json 2> gpurun_out/bench_host_post7.err || { tail gpurun_out/bench_host_post7.err; exit 1; }
cat gpurun_out/bench_host_post7.json
