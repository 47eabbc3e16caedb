# Round 3 kernel lab 4: partition knobs of the combined call (experiment library) + timeline
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/lab4
L=gpurun_out/lab4/lab.txt
: > $L
X=ITR_LIB=itrails_amd/libitrails_hip_exp.so
run() { timeout -k 10 120 env $X "$@" >> $L 2>&1 || { tail $L; exit 1; }; }
K="python scripts/kernel_lab.py --mean-block 2000 --which fv --reps 7"
run $K --tag default
run ITR_NO_MIXED=1 $K --tag nomixed
run ITR_VIT_LONG_FRAC=0.55 $K --tag lf55
run ITR_VIT_LONG_FRAC=0.65 $K --tag lf65
run ITR_VIT_RESERVE=48 $K --tag r48
run ITR_VIT_RESERVE=80 $K --tag r80
run ITR_URGENT_FRAC=0.35 $K --tag uf35
run ITR_URGENT_FRAC=0.4 $K --tag uf40
run ITR_FWD_RESERVE=16 $K --tag rf16
run ITR_FWD_RESERVE=32 $K --tag rf32
run ITR_VIT_LONG_FRAC=0.55 ITR_URGENT_FRAC=0.35 $K --tag lf55uf35
cat $L
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d gpurun_out/lab4/prof -o trace --output-format csv -- python3 scripts/prof_sweeps.py 3 fv > gpurun_out/lab4/prof.log 2>&1 || { tail gpurun_out/lab4/prof.log; exit 1; }
echo traced
