# GPU box: the register Gauss-Jordan inverse — dense + model tests, then config 5 and a build
# timeline.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r6m}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_dense.py tests/test_gpu_model.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
B="--cpu-1core-cols 0 --host-path 0"
timeout -k 10 300 python bench.py $B --mode optimize --steps 10 --warmup 3 > $O/opt55.json 2> $O/opt55.err || { tail $O/opt55.err; exit 1; }
python scripts/bench_line.py $O/opt55.json opt55
timeout -k 10 300 python bench.py $B --mode optimize --steps 10 --warmup 3 > $O/opt55b.json 2> $O/opt55b.err || { tail $O/opt55b.err; exit 1; }
python scripts/bench_line.py $O/opt55b.json opt55b
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/bt -o bt -- python scripts/build_timeline.py run 5 12 > $O/bt.log 2>&1 || { tail $O/bt.log; exit 1; }
f=$(find $O/bt -name "*kernel_trace.csv" | head -1)
python scripts/build_timeline.py analyse $f > $O/analysis.txt 2>&1
cp $f $O/kernel_trace.csv
rm -rf $O/bt
head -25 $O/analysis.txt
timeout -k 10 200 python scripts/build_stages.py 5 30 > $O/stages.txt 2>&1 && cat $O/stages.txt
