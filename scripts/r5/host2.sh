cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r5f}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_sweeps.py tests/test_gpu_distributed.py tests/test_gpu_rows.py -x -v -m gpu --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
ITR_HOST_TIMING=1 timeout -k 10 300 python scripts/host_wrap_timing.py 4 > $O/host_wrap.txt 2>&1 || { tail $O/host_wrap.txt; exit 1; }
cat $O/host_wrap.txt
timeout -k 10 300 python bench.py --cpu-1core-cols 0 > $O/bench_fv.json 2> $O/bench_fv.err || { tail $O/bench_fv.err; exit 1; }
python scripts/bench_line.py $O/bench_fv.json chr10
python -c "import json; print(json.load(open('$O/bench_fv.json'))['host_path'])"
echo done
