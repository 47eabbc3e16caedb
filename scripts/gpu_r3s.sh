# Round 3 lab: the CU partition with per-XCC masks (capi.cpp partition()); reserve / forward
# reserve / long-set fraction sweep on chr10, chr100 and the long-block workload
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r3s
L=gpurun_out/r3s/lab.txt
: > $L
X=ITR_LIB=itrails_amd/libitrails_hip_exp.so
run() { timeout -k 10 150 env $X "$@" >> $L 2>&1 || { tail $L; exit 1; }; }
K="python scripts/kernel_lab.py --mean-block 2000 --which fv --reps 9"
run python scripts/kernel_lab.py --mean-block 2000 --which vit,fv --reps 9 --check 1 --tag default
for r in 48 56 72 80; do run ITR_VIT_RESERVE=$r $K --tag r$r; done
for f in 16 32; do run ITR_FWD_RESERVE=$f $K --tag rf$f; done
for lf in 0.45 0.65; do run ITR_VIT_LONG_FRAC=$lf $K --tag lf$lf; done
run $K --tag default2
run python scripts/kernel_lab.py --mean-block 2000 --mbp 100 --which fv --reps 3 --tag chr100
run python scripts/kernel_lab.py --block-len 100000 --which fv,vit,fwd --reps 3 --check 1 --tag longblock
grep -v amdgpu.ids $L
