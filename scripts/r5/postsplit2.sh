# (7,7) posterior, split longest blocks: parity tests, then the split knobs (experiment build)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r5ps2}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu -k "post or 133 or 77" --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
B="--cpu-1core-cols 0 --host-path 0 --mode posterior --n-int 7"
timeout -k 10 400 python bench.py $B --steps 5 > $O/post77.json 2> $O/post77.err || { tail $O/post77.err; exit 1; }
python scripts/bench_line.py $O/post77.json post77
for cfg in ${CFGS:-"lo0.15:ITR_POST_BETA_LO=0.15" "lo0.25:ITR_POST_BETA_LO=0.25" "lo0.35:ITR_POST_BETA_LO=0.35" "f0.75:ITR_POST_BETA_FRAC=0.75" "nosplit:ITR_POST_BETA_FRAC=2"}; do
  IFS=: read lab envs <<< "$cfg"; envs=${envs//@/ }
  env $envs ITR_LIB=$PWD/itrails_amd/libitrails_hip_exp.so timeout -k 10 300 python bench.py $B --verify 0 --steps 3 > $O/$lab.json 2> $O/$lab.err || { tail $O/$lab.err; exit 1; }
  python scripts/bench_line.py $O/$lab.json $lab
done
echo done
