# Round 3 A/B on one box: mask variants of the planned partition (experiment library,
# ITR_MASK_MODE 0 per-XCC sets, 2 none, 3 bulk may share the long blocks' CUs) vs the
# round-start library; bench.py combined call, chr10 and chr100
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r3ab2
mkdir -p $O
L=$O/ab.txt
: > $L
B="--cpu-1core-cols 0 --host-path 0 --verify 0"
for i in 1 2; do
  for v in "exp 0" "exp 2" "exp 3" "r3start 0"; do
    set -- $v
    timeout -k 10 200 env ITR_LIB=itrails_amd/libitrails_hip_$1.so ITR_MASK_MODE=$2 python bench.py $B > $O/b.json 2> $O/b.err || { tail $O/b.err; exit 1; }
    python scripts/bench_line.py $O/b.json "chr10 $1 mode$2 $i" >> $L
  done
done
for v in "exp 0" "exp 2" "exp 3"; do
  set -- $v
  timeout -k 10 200 env ITR_LIB=itrails_amd/libitrails_hip_$1.so ITR_MASK_MODE=$2 python bench.py $B --workload chr100 --steps 3 > $O/b.json 2> $O/b.err || { tail $O/b.err; exit 1; }
  python scripts/bench_line.py $O/b.json "chr100 $1 mode$2" >> $L
done
grep -v amdgpu.ids $L
