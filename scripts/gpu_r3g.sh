# Round 3: SQ counters (two passes) + HBM bytes (FETCH_SIZE, WRITE_SIZE passes) of the sweep
# kernels: standalone forward, Viterbi, the combined call, the (7,7) posterior
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${TAG:-r3g}
O=gpurun_out/$T
mkdir -p $O/prof
P="python3 scripts/prof_sweeps.py 2 fwd,vit,fv,post"
timeout -s KILL 200 rocprofv3 --kernel-trace --stats -d $O/prof -o trace --output-format csv -- $P > $O/trace.log 2>&1 || { tail $O/trace.log; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA GRBM_GUI_ACTIVE -d $O/prof -o sq1 --output-format csv -- $P > $O/sq1.log 2>&1 || { tail $O/sq1.log; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_WAVES SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_FMA_F64 GRBM_GUI_ACTIVE -d $O/prof -o sq2 --output-format csv -- $P > $O/sq2.log 2>&1 || { tail $O/sq2.log; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -d $O/prof -o fetch --output-format csv -- $P > $O/fetch.log 2>&1 || { tail $O/fetch.log; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE -d $O/prof -o write --output-format csv -- $P > $O/write.log 2>&1 || { tail $O/write.log; exit 1; }
python scripts/pmc_summary.py $O/prof $O/pmc.json sweep wave_ hybrid trace combine > $O/pmc_summary.txt 2>&1
cat $O/pmc_summary.txt | head -80
