cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_dense.py tests/test_gpu_model.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_g2.log 2>&1 || { tail -30 gpurun_out/pytest_g2.log; exit 1; }
tail -1 gpurun_out/pytest_g2.log
timeout -k 10 300 python -u scripts/prof_build.py 5 3 > gpurun_out/prof_build.log 2>&1 || { tail -5 gpurun_out/prof_build.log; exit 1; }
grep -E "warm|enqueue" gpurun_out/prof_build.log
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_LDS_UNALIGNED_STALL -d gpurun_out/gpmc2 -o sq --output-format csv -- python3 scripts/prof_build.py 5 1 > gpurun_out/gpmc.log 2>&1 || { tail -5 gpurun_out/gpmc.log; exit 1; }
f=$(find gpurun_out/gpmc2 -name 'sq_counter_collection.csv' | head -1); python scripts/pmc_kernels.py $f pair_gemm
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/bprof2 -o bprof --output-format csv -- python3 scripts/prof_build.py 5 2 > gpurun_out/bprof.log 2>&1 || { tail -5 gpurun_out/bprof.log; exit 1; }
f=$(find gpurun_out/bprof2 -name '*kernel_stats.csv' | head -1); head -4 $f | cut -c1-160
