# Round 3: sweep parity tests, then the default bench twice, then SQ counters of the forward
# and Viterbi kernels (separate calls via scripts/prof_sweeps.py).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${TAG:-r3c}
mkdir -p gpurun_out/$T
timeout -k 10 300 python -u -m pytest tests/test_gpu_sweeps.py tests/test_gpu_fullsize.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/$T/pytest.log 2>&1 || { tail -30 gpurun_out/$T/pytest.log; exit 1; }
tail -1 gpurun_out/$T/pytest.log
for i in 1 2; do
timeout -k 10 300 python bench.py --verify 0 --cpu-1core-cols 0 --host-path 0 --steps 10 > gpurun_out/$T/bench$i.json 2> gpurun_out/$T/bench$i.err || { tail gpurun_out/$T/bench$i.err; exit 1; }
python scripts/bench_line.py gpurun_out/$T/bench$i.json run$i
done
if [ -n "$PMC" ]; then
P="python3 scripts/prof_sweeps.py"
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d gpurun_out/$T/prof -o trace --output-format csv -- $P > gpurun_out/$T/prof_trace.log 2>&1 || { tail gpurun_out/$T/prof_trace.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA GRBM_GUI_ACTIVE -d gpurun_out/$T/prof -o sq1 --output-format csv -- $P > gpurun_out/$T/sq1.log 2>&1 || { tail gpurun_out/$T/sq1.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_WAVES SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_FMA_F64 GRBM_GUI_ACTIVE -d gpurun_out/$T/prof -o sq2 --output-format csv -- $P > gpurun_out/$T/sq2.log 2>&1 || { tail gpurun_out/$T/sq2.log; exit 1; }
python scripts/pmc_summary.py gpurun_out/$T/prof gpurun_out/$T/pmc.json sweep wave_vit hybrid trace
fi
