# Round 4: is the (7,7) posterior bound by its longest blocks?  Same 10 Mbp as equal
# 2,000-column blocks vs the chr10 layout (longest 18,377); urgent fraction sweep
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r4pc}
mkdir -p $O
B="--cpu-1core-cols 0 --host-path 0 --mode posterior --n-int 7 --steps 3 --verify 0"
timeout -k 10 300 python bench.py $B --block-len 2000 > $O/eq2k.json 2> $O/eq2k.err || { tail $O/eq2k.err; exit 1; }
python scripts/bench_line.py $O/eq2k.json "post77 equal 2k blocks"
timeout -k 10 300 python bench.py $B > $O/base.json 2> $O/base.err || { tail $O/base.err; exit 1; }
python scripts/bench_line.py $O/base.json "post77 chr10 layout"
for F in 0.3 0.7; do
  ITR_LIB=itrails_amd/libitrails_hip_exp.so ITR_POST_URGENT_FRAC=$F timeout -k 10 300 python bench.py $B > $O/f$F.json 2> $O/f$F.err || { tail $O/f$F.err; exit 1; }
  python scripts/bench_line.py $O/f$F.json "post77 pfrac $F"
done
echo done
