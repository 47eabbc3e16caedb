# Round 3 lab: planner constants after the SE-balanced partition and the early traceback
# (experiment library: ITR_WAVE_LAT, ITR_BULK_CU), bench.py combined call, chr10, alternated
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r3k2
mkdir -p $O
L=$O/lab.txt
: > $L
B="--cpu-1core-cols 0 --host-path 0 --verify 0 --steps 8"
for i in 1 2; do
  for v in "0.8 0.18" "0.7 0.18" "0.9 0.18" "0.8 0.165" "0.8 0.195" "0.75 0.17"; do
    set -- $v
    timeout -k 10 200 env ITR_LIB=itrails_amd/libitrails_hip_exp.so ITR_WAVE_LAT=$1e-6 ITR_BULK_CU=$2e-6 python bench.py $B > $O/b.json 2> $O/b.err || { tail $O/b.err; exit 1; }
    python scripts/bench_line.py $O/b.json "chr10 wlat$1 bulk$2 $i" >> $L
  done
done
grep -v amdgpu.ids $L
