# (7,7) posterior with the longest blocks' beta sweep beside their forward one: parity tests,
# the post77 line, then the split threshold (experiment build)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r5ps}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu -k "post or 133 or 77" --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
B="--cpu-1core-cols 0 --host-path 0 --mode posterior --n-int 7 --steps 5"
timeout -k 10 400 python bench.py $B > $O/post77.json 2> $O/post77.err || { tail $O/post77.err; exit 1; }
python scripts/bench_line.py $O/post77.json post77
for f in ${FRACS:-0.5 0.6 0.75 0.9 2}; do
  ITR_POST_BETA_FRAC=$f ITR_LIB=$PWD/itrails_amd/libitrails_hip_exp.so timeout -k 10 300 python bench.py $B --verify 0 --steps 3 > $O/f$f.json 2> $O/f$f.err || { tail $O/f$f.err; exit 1; }
  python scripts/bench_line.py $O/f$f.json frac$f
done
echo done
