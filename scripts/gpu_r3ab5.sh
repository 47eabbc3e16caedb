# Round 3 A/B on one box: planner bulk-cost constant sweep (per-XCC masks) vs round start
# Round 3 A/B: SE-balanced reserved sets; planner bulk-cost sweep; rounding to XCC (8) or SE (32) sets
export TMPDIR=/tmp
O=gpurun_out/r3ab5
mkdir -p $O
L=$O/ab.txt
: > $L
B="--cpu-1core-cols 0 --host-path 0 --verify 0 --steps 8"
for i in 1 2; do
  for v in "exp 0.15" "exp 0.165" "exp 0.18" "exp 0.195" "r3start 0" "exp 0.15 1" "exp 0.18 1"; do
    set -- $v
    timeout -k 10 200 env ITR_LIB=itrails_amd/libitrails_hip_$1.so ITR_BULK_CU=$2e-6 ${3:+ITR_SE_ROUND=1} python bench.py $B > $O/b.json 2> $O/b.err || { tail $O/b.err; exit 1; }
    python scripts/bench_line.py $O/b.json "chr10 $1 bulk$2 se$3 $i" >> $L
  done
done
for v in "0.15" "0.18"; do
  timeout -k 10 200 env ITR_LIB=itrails_amd/libitrails_hip_exp.so ITR_BULK_CU=${v}e-6 python bench.py $B --workload chr100 --steps 3 > $O/b.json 2> $O/b.err || { tail $O/b.err; exit 1; }
  python scripts/bench_line.py $O/b.json "chr100 bulk$v" >> $L
  timeout -k 10 200 env ITR_LIB=itrails_amd/libitrails_hip_exp.so ITR_BULK_CU=${v}e-6 python bench.py $B --mbp 12.5 > $O/b.json 2> $O/b.err || { tail $O/b.err; exit 1; }
  python scripts/bench_line.py $O/b.json "chr12.5 bulk$v" >> $L
done
grep -v amdgpu.ids $L
