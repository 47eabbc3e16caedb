# Round 3, first pass: FP64 MFMA / VALU co-issue micro, counter list, GPU tests, default
# bench, SQ counter passes over the chr10 step (one rocprofv3 --pmc pass per counter set).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r3a
:
:
timeout -k 10 60 rocprofv3 -L > gpurun_out/r3a/counters.txt 2>&1 || { tail gpurun_out/r3a/counters.txt; exit 1; }
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/r3a/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/r3a/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/r3a/pytest_gpu.log
timeout -k 10 300 python bench.py > gpurun_out/r3a/bench.json 2> gpurun_out/r3a/bench.err || { tail gpurun_out/r3a/bench.err; exit 1; }
cat gpurun_out/r3a/bench.json
B="python3 bench.py --steps 2 --warmup 1 --verify 0 --cpu-1core-cols 0 --host-path 0"
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d gpurun_out/r3a/prof -o trace --output-format csv -- $B > gpurun_out/r3a/prof_trace.log 2>&1 || { tail gpurun_out/r3a/prof_trace.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS -d gpurun_out/r3a/prof -o sq1 --output-format csv -- $B > gpurun_out/r3a/sq1.log 2>&1 || { tail gpurun_out/r3a/sq1.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_ACTIVE_INST_MFMA SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_WAVES GRBM_GUI_ACTIVE -d gpurun_out/r3a/prof -o sq2 --output-format csv -- $B > gpurun_out/r3a/sq2.log 2>&1 || { tail gpurun_out/r3a/sq2.log; exit 1; }
echo done
