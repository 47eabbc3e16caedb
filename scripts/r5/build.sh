# model-build checks and timing: dense / model GPU tests, the config-5 bench, the build's
# cProfile and kernel trace, and the drop-in host path's stage times
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r5c}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_dense.py tests/test_gpu_model.py tests/test_gpu_distributed.py -x -v -m gpu --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python bench.py --cpu-1core-cols 0 --host-path 0 --mode optimize --steps 10 --warmup 3 > $O/opt55.json 2> $O/opt55.err || { tail $O/opt55.err; exit 1; }
python scripts/bench_line.py $O/opt55.json opt55
timeout -k 10 300 python scripts/prof_build.py 5 8 > $O/prof_build.log 2>&1 || { tail $O/prof_build.log; exit 1; }
head -12 $O/prof_build.log
timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d $O/bprof -o trace --output-format csv -- python3 scripts/prof_build.py 5 8 > $O/bprof.log 2>&1 || { tail $O/bprof.log; exit 1; }
timeout -k 10 300 python scripts/host_path_timing.py 4 > $O/host_path.txt 2>&1 || { tail $O/host_path.txt; exit 1; }
cat $O/host_path.txt
echo done
