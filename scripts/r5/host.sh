# GPU tests, smoke, host-path stage times, the lone Viterbi step's stage cycles (diag build)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r5d}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python scripts/host_path_timing.py 4 > $O/host_path.txt 2>&1 || { tail $O/host_path.txt; exit 1; }
cat $O/host_path.txt
timeout -k 10 300 python bench.py --cpu-1core-cols 0 > $O/bench_fv.json 2> $O/bench_fv.err || { tail $O/bench_fv.err; exit 1; }
python scripts/bench_line.py $O/bench_fv.json chr10
python -c "import json; print(json.load(open('$O/bench_fv.json'))['host_path'])"
ITR_LIB=$PWD/itrails_amd/libitrails_hip_diag.so timeout -k 10 300 python scripts/vit_stages.py > $O/vit_stages.txt 2>&1 || { tail $O/vit_stages.txt; exit 1; }
cat $O/vit_stages.txt
echo done
