# GPU box, round 6 final pass, one lease and one library: every GPU test + smoke, the default
# bench line, a rocprofv3 kernel trace of the SAME default command (20 timed steps after 10
# warmup steps), FETCH_SIZE / WRITE_SIZE passes of it (-> fv_call_traffic.json, tied to the
# library hash), SQ / matrix-core / HBM counters of every sweep entry point, then every other
# BASELINE line; outputs under gpurun_out/$TAG.  Each GPU step has its own time limit and the
# script stops at the first failure.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${TAG:-r6z}
O=gpurun_out/$T
mkdir -p $O/prof $O/sq
if [ -z "$SKIP_TESTS" ]; then
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
fi
timeout -k 10 400 python bench.py > $O/bench_fv.json 2> $O/bench_fv.err || { tail $O/bench_fv.err; exit 1; }
python scripts/bench_line.py $O/bench_fv.json chr10
P="python3 bench.py --verify 0 --cpu-1core-cols 0 --host-path 0"
timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d $O/prof -o trace --output-format csv -- $P > $O/prof_trace.log 2>&1 || { tail $O/prof_trace.log; exit 1; }
tail -1 $O/prof_trace.log
P3="python3 bench.py --steps 3 --warmup 1 --verify 0 --cpu-1core-cols 0 --host-path 0"
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE -d $O/prof -o pmc_fetch --output-format csv -- $P3 > $O/prof_fetch.log 2>&1 || { tail $O/prof_fetch.log; exit 1; }
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE -d $O/prof -o pmc_write --output-format csv -- $P3 > $O/prof_write.log 2>&1 || { tail $O/prof_write.log; exit 1; }
python scripts/fv_traffic.py $O/prof $O/fv_call_traffic.json > /dev/null
S="python3 scripts/prof_sweeps.py 2 fwd,vit,fv,post,post5"
timeout -s KILL 200 rocprofv3 --kernel-trace --stats -d $O/sq -o trace --output-format csv -- $S > $O/sq_trace.log 2>&1 || { tail $O/sq_trace.log; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA GRBM_GUI_ACTIVE -d $O/sq -o sq1 --output-format csv -- $S > $O/sq1.log 2>&1 || { tail $O/sq1.log; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_WAVES SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_FMA_F64 GRBM_GUI_ACTIVE -d $O/sq -o sq2 --output-format csv -- $S > $O/sq2.log 2>&1 || { tail $O/sq2.log; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -d $O/sq -o fetch --output-format csv -- $S > $O/sqf.log 2>&1 || { tail $O/sqf.log; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE -d $O/sq -o write --output-format csv -- $S > $O/sqw.log 2>&1 || { tail $O/sqw.log; exit 1; }
python scripts/pmc_summary.py $O/sq $O/pmc.json sweep wave_ hybrid trace combine prune group > $O/pmc_summary.txt 2>&1
echo profiles done
