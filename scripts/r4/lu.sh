# Round 4: LDS-resident LU panel: dense + model GPU tests, build profile, optimize line
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r4lu}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_dense.py tests/test_gpu_model.py -x -q -m gpu --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 200 python3 scripts/prof_build.py 5 8 > $O/prof_build.log 2>&1 || { tail $O/prof_build.log; exit 1; }
head -12 $O/prof_build.log
timeout -k 10 300 python bench.py --cpu-1core-cols 0 --host-path 0 --mode optimize --steps 10 --warmup 3 > $O/opt.json 2> $O/opt.err || { tail $O/opt.err; exit 1; }
python scripts/bench_line.py $O/opt.json optimize
echo done
