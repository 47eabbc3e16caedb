cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_LDS_UNALIGNED_STALL -d gpurun_out/gpmc -o sq --output-format csv -- python3 scripts/prof_build.py 5 1 > gpurun_out/gpmc.log 2>&1 || { tail -5 gpurun_out/gpmc.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE SQ_INSTS_LDS -d gpurun_out/gpmc -o fetch --output-format csv -- python3 scripts/prof_build.py 5 1 > gpurun_out/gpmc2.log 2>&1 || { tail -5 gpurun_out/gpmc2.log; exit 1; }
f=$(find gpurun_out/gpmc -name 'sq_counter_collection.csv' | head -1); python scripts/pmc_kernels.py $f pair_gemm
f=$(find gpurun_out/gpmc -name 'fetch_counter_collection.csv' | head -1); python scripts/pmc_kernels.py $f pair_gemm
