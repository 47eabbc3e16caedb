# Round 3 kernel lab: standalone sweep throughput (CU-ns per column) on short and chr10 blocks,
# with experiment knobs (experiment library).
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/lab1
L=gpurun_out/lab1/lab.txt
: > $L
run() { timeout -k 10 120 env "$@" >> $L 2>&1 || { tail $L; exit 1; }; }
run ITR_LIB=itrails_amd/libitrails_hip_exp.so python scripts/kernel_lab.py --mean-block 250 --which fwd,vit --tag short
run ITR_LIB=itrails_amd/libitrails_hip_exp.so ITR_HYB_PER_CU=3 python scripts/kernel_lab.py --mean-block 250 --which fwd --tag short_percu3
run ITR_LIB=itrails_amd/libitrails_hip_exp.so ITR_HYB_PER_CU=1 python scripts/kernel_lab.py --mean-block 250 --which fwd --tag short_percu1
run ITR_LIB=itrails_amd/libitrails_hip_exp.so ITR_NO_MFMA=1 python scripts/kernel_lab.py --mean-block 250 --which fwd --tag short_valu
run ITR_LIB=itrails_amd/libitrails_hip_exp.so python scripts/kernel_lab.py --mean-block 2000 --which fwd,vit,fv --tag chr10
run ITR_LIB=itrails_amd/libitrails_hip_exp.so ITR_NO_WAVE=1 python scripts/kernel_lab.py --mean-block 250 --which vit --tag short_9wave
cat $L
