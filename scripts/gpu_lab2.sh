# Round 3 kernel lab 2: the per-wave matrix-core forward (ITR_WAVE_FWD, experiment library)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/lab2
L=gpurun_out/lab2/lab.txt
: > $L
run() { timeout -k 10 120 env "$@" >> $L 2>&1 || { tail $L; exit 1; }; }
X=ITR_LIB=itrails_amd/libitrails_hip_exp.so
run $X ITR_WAVE_FWD=1 python scripts/kernel_lab.py --mean-block 250 --which fwd --tag short_wavefwd --check 1
run $X python scripts/kernel_lab.py --mean-block 250 --which fwd --tag short_hybrid
run $X ITR_WAVE_FWD=1 python scripts/kernel_lab.py --mean-block 2000 --which fwd --tag chr10_wavefwd --check 1
run $X ITR_WAVE_FWD=1 python scripts/kernel_lab.py --mean-block 250 --mbp 2 --which fwd --tag short2_wavefwd
cat $L
