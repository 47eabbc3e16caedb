# Round 3 lab: CU masks: per-XCC (0), round-2 pattern (1, no effective mask), none (2); mixed grid
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r3t
L=gpurun_out/r3t/lab.txt
: > $L
X=ITR_LIB=itrails_amd/libitrails_hip_exp.so
run() { timeout -k 10 150 env $X "$@" >> $L 2>&1 || { tail $L; exit 1; }; }
K="python scripts/kernel_lab.py --mean-block 2000 --which fv --reps 9"
for i in 1 2; do
run ITR_MASK_MODE=0 $K --tag m0_$i
run ITR_MASK_MODE=1 $K --tag m1_$i
run ITR_MASK_MODE=2 $K --tag m2_$i
run ITR_MASK_MODE=2 ITR_MIX_CUS=256 $K --tag m2_mix256_$i
run ITR_MASK_MODE=0 ITR_VIT_LONG_FRAC=0.45 ITR_VIT_RESERVE=72 $K --tag m0_lf45_r72_$i
run ITR_MASK_MODE=0 ITR_VIT_LONG_FRAC=0.4 ITR_VIT_RESERVE=80 ITR_FWD_RESERVE=32 $K --tag m0_lf40_r80_rf32_$i
done
run ITR_MASK_MODE=1 python scripts/kernel_lab.py --mean-block 2000 --mbp 100 --which fv --reps 3 --tag chr100_m1
run ITR_MASK_MODE=2 python scripts/kernel_lab.py --mean-block 2000 --mbp 100 --which fv --reps 3 --tag chr100_m2
run ITR_MASK_MODE=1 python scripts/kernel_lab.py --block-len 100000 --which fv --reps 3 --tag longblock_m1
run ITR_MASK_MODE=2 python scripts/kernel_lab.py --block-len 100000 --which fv --reps 3 --tag longblock_m2
grep -v amdgpu.ids $L
