# Round 3 A/B on one box: the current library vs the round-start library (ITR_LIB), bench.py
# (side stream, combined call per step) and the kernel lab (default stream), alternated
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r3ab
mkdir -p $O
L=$O/ab.txt
: > $L
B="--cpu-1core-cols 0 --host-path 0 --verify 0"
for i in 1 2; do
  for lib in libitrails_hip.so libitrails_hip_r3start.so; do
    timeout -k 10 200 env ITR_LIB=itrails_amd/$lib python bench.py $B > $O/b.json 2> $O/b.err || { tail $O/b.err; exit 1; }
    python scripts/bench_line.py $O/b.json "bench $lib $i" >> $L
    timeout -k 10 200 env ITR_LIB=itrails_amd/$lib python scripts/kernel_lab.py --mean-block 2000 --which vit,fv --reps 9 --tag "lab $lib $i" >> $L 2>&1 || { tail $L; exit 1; }
  done
done
timeout -k 10 200 env ITR_LIB=itrails_amd/libitrails_hip.so python bench.py $B --workload chr100 --steps 3 > $O/b.json 2> $O/b.err && python scripts/bench_line.py $O/b.json "chr100 current" >> $L
timeout -k 10 200 env ITR_LIB=itrails_amd/libitrails_hip_r3start.so python bench.py $B --workload chr100 --steps 3 > $O/b.json 2> $O/b.err && python scripts/bench_line.py $O/b.json "chr100 r3start" >> $L
grep -v amdgpu.ids $L
