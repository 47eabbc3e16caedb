# Round 4: bound-pruned per-wave Viterbi: sweep + full-size GPU tests, fv / vit bench lines
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r4p}
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_sweeps.py tests/test_gpu_fullsize.py -x -v -m gpu --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
B="--cpu-1core-cols 0 --host-path 0"
timeout -k 10 300 python bench.py $B > $O/fv.json 2> $O/fv.err || { tail $O/fv.err; exit 1; }
python scripts/bench_line.py $O/fv.json chr10
timeout -k 10 300 python bench.py $B --mode vit > $O/vit.json 2> $O/vit.err || { tail $O/vit.err; exit 1; }
python scripts/bench_line.py $O/vit.json vit
echo done
