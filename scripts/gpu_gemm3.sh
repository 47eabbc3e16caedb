cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for lib in libitrails_hip.so libitrails_hip_tk32.so; do
export ITR_LIB=$PWD/itrails_amd/$lib
timeout -k 10 400 python -u -m pytest tests/test_gpu_dense.py tests/test_gpu_model.py -x -q -m gpu -k "vanloan or trans_emiss_calc_matches" --timeout 300 --timeout-method thread > gpurun_out/pytest_g3.log 2>&1 || { tail -30 gpurun_out/pytest_g3.log; exit 1; }
echo $lib; tail -1 gpurun_out/pytest_g3.log
timeout -k 10 300 python -u scripts/prof_build.py 5 3 > gpurun_out/prof_build.log 2>&1 || { tail -5 gpurun_out/prof_build.log; exit 1; }
grep -E "warm" gpurun_out/prof_build.log
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_INST_ANY -d gpurun_out/gpmc3_$lib -o sq --output-format csv -- python3 scripts/prof_build.py 5 1 > gpurun_out/gpmc.log 2>&1 || { tail -5 gpurun_out/gpmc.log; exit 1; }
f=$(find gpurun_out/gpmc3_$lib -name 'sq_counter_collection.csv' | head -1); python scripts/pmc_kernels.py $f pair_gemm
done
