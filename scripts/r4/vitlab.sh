# Viterbi-only long-set size lab (experiment library, ITR_VIT_NLONG_V), chr10, vit mode
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r4m}
mkdir -p $O
: > $O/lab.txt
B="--cpu-1core-cols 0 --host-path 0 --verify 0 --mode vit --steps 8"
for k in 0 30 59 80 100 124 150; do
  timeout -k 10 200 env ITR_LIB=itrails_amd/libitrails_hip_exp.so ITR_VIT_NLONG_V=$k python bench.py $B > $O/b.json 2> $O/b.err || { tail $O/b.err; exit 1; }
  python scripts/bench_line.py $O/b.json "nlong_v $k" >> $O/lab.txt
done
grep -v amdgpu.ids $O/lab.txt
