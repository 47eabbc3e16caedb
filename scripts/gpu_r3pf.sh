# Round 3 lab: (7,7) posterior, VALU/matrix-core split fraction (experiment library,
# ITR_POST_URGENT_FRAC) after the matrix-core chain change
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r3pf
mkdir -p $O
L=$O/lab.txt
: > $L
B="--cpu-1core-cols 0 --host-path 0 --verify 0 --steps 4"
for f in 0.5 0.35 0.42 0.6 0.75 1.5; do
  timeout -k 10 200 env ITR_LIB=itrails_amd/libitrails_hip_exp.so ITR_POST_URGENT_FRAC=$f python bench.py $B --mode posterior --n-int 7 > $O/b.json 2> $O/b.err || { tail $O/b.err; exit 1; }
  python scripts/bench_line.py $O/b.json "post77 pfrac $f" >> $L
done
grep -v amdgpu.ids $L
