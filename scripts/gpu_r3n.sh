# Round 3 lab: Viterbi with K blocks per wavefront (experiment library, ITR_VIT_SLOTS=K) vs
# the one-block-per-wave layout; standalone itr_viterbi, short blocks and chr10, paths checked
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r3n
L=gpurun_out/r3n/lab.txt
: > $L
X=ITR_LIB=itrails_amd/libitrails_hip_exp.so
run() { timeout -k 10 150 env $X "$@" >> $L 2>&1 || { tail $L; exit 1; }; }
for mb in 300 2000; do
  run python scripts/kernel_lab.py --mean-block $mb --which vit --reps 7 --check 1 --tag "k1_mb$mb"
  for k in 2 3 4; do
    run ITR_VIT_SLOTS=$k python scripts/kernel_lab.py --mean-block $mb --which vit --reps 7 --check 1 --tag "k${k}_mb$mb"
  done
done
grep -v amdgpu.ids $L
