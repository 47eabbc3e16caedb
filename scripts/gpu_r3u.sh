# Round 3 lab: per-XCC partition sweep (reserve, long fraction, forward reserve) + bulk
# occupancy probe; longblock with unmasked streams
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r3u
L=gpurun_out/r3u/lab.txt
: > $L
X=ITR_LIB=itrails_amd/libitrails_hip_exp.so
run() { timeout -k 10 150 env $X "$@" >> $L 2>&1 || { tail $L; exit 1; }; }
K="python scripts/kernel_lab.py --mean-block 2000 --which fv --reps 9"
run python scripts/kernel_lab.py --mean-block 2000 --which vit,fv --reps 9 --check 1 --tag default
for i in 1 2; do
for c in "0.45 72" "0.4 72" "0.4 80" "0.5 72" "0.45 64" "0.45 80" "0.35 88"; do
  set -- $c
  run ITR_VIT_LONG_FRAC=$1 ITR_VIT_RESERVE=$2 $K --tag "lf$1_r$2_$i"
done
run ITR_FWD_RESERVE=20 $K --tag "rf20_$i"
run ITR_FWD_RESERVE=34 $K --tag "rf34_$i"
done
run python scripts/kernel_lab.py --mean-block 2000 --mbp 100 --which fv --reps 3 --tag chr100
run python scripts/kernel_lab.py --block-len 100000 --which fv --reps 3 --check 1 --tag longblock
grep -v amdgpu.ids $L
