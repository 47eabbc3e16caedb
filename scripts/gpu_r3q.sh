# Round 3 lab: reserved CUs stealing from the mixed queue vs not (experiment library), same box
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r3q
L=gpurun_out/r3q/lab.txt
: > $L
X=ITR_LIB=itrails_amd/libitrails_hip_exp.so
run() { timeout -k 10 150 env $X "$@" >> $L 2>&1 || { tail $L; exit 1; }; }
K="python scripts/kernel_lab.py --mean-block 2000 --which fv --reps 15"
for i in 1 2 3; do
  run $K --tag steal_$i
  run ITR_NO_STEAL=1 $K --tag nosteal_$i
done
run python scripts/kernel_lab.py --mean-block 2000 --mbp 100 --which fv --reps 5 --tag chr100_steal
run ITR_NO_STEAL=1 python scripts/kernel_lab.py --mean-block 2000 --mbp 100 --which fv --reps 5 --tag chr100_nosteal
grep -v amdgpu.ids $L
