# GPU box: every GPU test, smoke, the default bench, then (unless QUICK) the other BASELINE
# configs' lines, a rocprofv3 kernel trace + FETCH_SIZE / WRITE_SIZE passes of the default
# bench (-> fv_call_traffic.json with the library hash); outputs under gpurun_out/$TAG.
# Every GPU step has its own time limit; the script stops at the first failure.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${TAG:-r5}
O=gpurun_out/$T
mkdir -p $O/prof
if [ -z "$SKIP_TESTS" ]; then
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
fi
timeout -k 10 400 python bench.py > $O/bench_fv.json 2> $O/bench_fv.err || { tail $O/bench_fv.err; exit 1; }
python scripts/bench_line.py $O/bench_fv.json chr10
B="--cpu-1core-cols 0 --host-path 0"
P="python3 bench.py --steps 3 --warmup 1 --verify 0 $B"
timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d $O/prof -o trace --output-format csv -- $P > $O/prof_trace.log 2>&1 || { tail $O/prof_trace.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/prof -o pmc_fetch --output-format csv -- $P > $O/prof_fetch.log 2>&1 || { tail $O/prof_fetch.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/prof -o pmc_write --output-format csv -- $P > $O/prof_write.log 2>&1 || { tail $O/prof_write.log; exit 1; }
python scripts/fv_traffic.py $O/prof $O/fv_call_traffic.json > /dev/null
[ -n "$QUICK" ] && { echo done; exit 0; }
# SQ / matrix-core / HBM counters of the sweep kernels, one configuration per entry point
S="python3 scripts/prof_sweeps.py 2 fwd,vit,fv,post"
mkdir -p $O/sq
timeout -s KILL 200 rocprofv3 --kernel-trace --stats -d $O/sq -o trace --output-format csv -- $S > $O/sq_trace.log 2>&1 || { tail $O/sq_trace.log; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA GRBM_GUI_ACTIVE -d $O/sq -o sq1 --output-format csv -- $S > $O/sq1.log 2>&1 || { tail $O/sq1.log; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_WAVES SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_FMA_F64 GRBM_GUI_ACTIVE -d $O/sq -o sq2 --output-format csv -- $S > $O/sq2.log 2>&1 || { tail $O/sq2.log; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -d $O/sq -o fetch --output-format csv -- $S > $O/sqf.log 2>&1 || { tail $O/sqf.log; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE -d $O/sq -o write --output-format csv -- $S > $O/sqw.log 2>&1 || { tail $O/sqw.log; exit 1; }
python scripts/pmc_summary.py $O/sq $O/pmc.json sweep wave_ hybrid trace combine prune > $O/pmc_summary.txt 2>&1
timeout -k 10 300 python bench.py $B --mode vit > $O/vit.json 2> $O/vit.err || { tail $O/vit.err; exit 1; }
python scripts/bench_line.py $O/vit.json vit
timeout -k 10 300 python bench.py $B --workload chr100 --steps 3 --project-shards 8 > $O/chr100.json 2> $O/chr100.err || { tail $O/chr100.err; exit 1; }
python scripts/bench_line.py $O/chr100.json chr100
timeout -k 10 300 python bench.py $B --block-len 100000 --steps 5 > $O/lb.json 2> $O/lb.err || { tail $O/lb.err; exit 1; }
python scripts/bench_line.py $O/lb.json longblock
timeout -k 10 400 python bench.py $B --mode posterior --n-int 7 --steps 5 > $O/post77.json 2> $O/post77.err || { tail $O/post77.err; exit 1; }
python scripts/bench_line.py $O/post77.json post77
timeout -k 10 300 python bench.py $B --n-int 7 > $O/fv77.json 2> $O/fv77.err || { tail $O/fv77.err; exit 1; }
python scripts/bench_line.py $O/fv77.json fv77
timeout -k 10 300 python bench.py $B --model introgression > $O/fvint.json 2> $O/fvint.err || { tail $O/fvint.err; exit 1; }
python scripts/bench_line.py $O/fvint.json fv_intro95
timeout -k 10 300 python bench.py $B --mode optimize --steps 10 --warmup 3 > $O/opt55.json 2> $O/opt55.err || { tail $O/opt55.err; exit 1; }
python scripts/bench_line.py $O/opt55.json opt55
timeout -k 10 300 python bench.py $B --dist 1 --backend nccl > $O/rccl1.json 2> $O/rccl1.err || { tail $O/rccl1.err; exit 1; }
python scripts/bench_line.py $O/rccl1.json chr10_rccl_world1

timeout -k 10 400 python bench.py $B --mode posterior --n-int 5 --steps 5 > $O/post55.json 2> $O/post55.err || { tail $O/post55.err; exit 1; }
python scripts/bench_line.py $O/post55.json post55
echo done
