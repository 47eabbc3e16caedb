# Round 3 kernel lab 5: reserved CUs / forward VALU CUs with the 0.55 long set (experiment lib)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/lab5
L=gpurun_out/lab5/lab.txt
: > $L
X=ITR_LIB=itrails_amd/libitrails_hip_exp.so
run() { timeout -k 10 120 env $X "$@" >> $L 2>&1 || { tail $L; exit 1; }; }
K="python scripts/kernel_lab.py --mean-block 2000 --which fv --reps 7"
run $K --tag default
run ITR_VIT_RESERVE=48 $K --tag r48
run ITR_VIT_RESERVE=56 $K --tag r56
run ITR_VIT_RESERVE=72 $K --tag r72
run ITR_FWD_RESERVE=16 $K --tag rf16
run ITR_FWD_RESERVE=20 $K --tag rf20
run ITR_VIT_RESERVE=56 ITR_FWD_RESERVE=20 $K --tag r56rf20
run ITR_VIT_LONG_FRAC=0.6 $K --tag lf60
run ITR_VIT_LONG_FRAC=0.5 $K --tag lf50
run $K --tag default2
grep -v amdgpu.ids $L
