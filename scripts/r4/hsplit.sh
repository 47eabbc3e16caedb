# Round 4: the hybrid posterior's concurrent split (product) vs the two-phase hybrid
# (ITR_POST_HSPLIT=0, experiment library): sweep + full-size GPU tests, (7,7) posterior
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r4hs}
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_sweeps.py tests/test_gpu_fullsize.py -x -q -m gpu --timeout 250 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
B="--cpu-1core-cols 0 --host-path 0 --mode posterior --n-int 7 --steps 5"
timeout -k 10 300 python bench.py $B > $O/split.json 2> $O/split.err || { tail $O/split.err; exit 1; }
python scripts/bench_line.py $O/split.json "post77 split"
ITR_LIB=itrails_amd/libitrails_hip_exp.so ITR_POST_HSPLIT=0 timeout -k 10 300 python bench.py $B --verify 0 > $O/two.json 2> $O/two.err || { tail $O/two.err; exit 1; }
python scripts/bench_line.py $O/two.json "post77 two-phase"
echo done
