# Round 3 A/B on one box: planner bulk-cost constant (ITR_BULK_CU) x mask mode vs the
# round-start library; bench.py combined call timer (fv), chr10; chr100 once
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r3ab3
mkdir -p $O
L=$O/ab.txt
: > $L
B="--cpu-1core-cols 0 --host-path 0 --verify 0 --steps 8"
for i in 1 2; do
  for v in "exp 0 0.21" "exp 2 0.21" "exp 0 0.25" "exp 2 0.25" "exp 0 0.18" "r3start 0 0"; do
    set -- $v
    timeout -k 10 200 env ITR_LIB=itrails_amd/libitrails_hip_$1.so ITR_MASK_MODE=$2 ITR_BULK_CU=$3e-6 python bench.py $B > $O/b.json 2> $O/b.err || { tail $O/b.err; exit 1; }
    python scripts/bench_line.py $O/b.json "chr10 $1 mode$2 bulk$3 $i" >> $L
  done
done
for v in "exp 0 0.21" "exp 2 0.21"; do
  set -- $v
  timeout -k 10 200 env ITR_LIB=itrails_amd/libitrails_hip_$1.so ITR_MASK_MODE=$2 ITR_BULK_CU=$3e-6 python bench.py $B --workload chr100 --steps 3 > $O/b.json 2> $O/b.err || { tail $O/b.err; exit 1; }
  python scripts/bench_line.py $O/b.json "chr100 $1 mode$2 bulk$3" >> $L
done
grep -v amdgpu.ids $L
