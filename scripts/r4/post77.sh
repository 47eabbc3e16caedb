# Round 4: (7,7) posterior with one (product) vs two matrix-core groups per workgroup
# (experiment configuration ITR_MCFG=7), and the optimize line after the vectorised tables
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r4pa}
mkdir -p $O
B="--cpu-1core-cols 0 --host-path 0"
timeout -k 10 300 python bench.py $B --mode optimize --steps 10 --warmup 3 > $O/opt.json 2> $O/opt.err || { tail $O/opt.err; exit 1; }
python scripts/bench_line.py $O/opt.json optimize
timeout -k 10 300 python bench.py $B --mode posterior --n-int 7 --steps 5 --verify 0 > $O/p_base.json 2> $O/p_base.err || { tail $O/p_base.err; exit 1; }
python scripts/bench_line.py $O/p_base.json "post77 base"
for M in 7; do
  ITR_LIB=itrails_amd/libitrails_hip_exp.so ITR_MCFG=$M timeout -k 10 300 python bench.py $B --mode posterior --n-int 7 --steps 5 > $O/p_m$M.json 2> $O/p_m$M.err || { tail $O/p_m$M.err; exit 1; }
  python scripts/bench_line.py $O/p_m$M.json "post77 mcfg $M"
done
echo done
