# Round 3: per-wave Viterbi lane mapping (bank-conflict-free partial writes): parity, lab
# throughput on short blocks and on chr10, bank-conflict counters of the Viterbi call
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r3m}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_sweeps.py tests/test_gpu_fullsize.py -x -q -m gpu --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
L=$O/lab.txt
timeout -k 10 120 python scripts/kernel_lab.py --mean-block 300 --which vit,fwd,fv --reps 7 --tag short300 > $L 2>&1 || { tail $L; exit 1; }
timeout -k 10 120 python scripts/kernel_lab.py --mean-block 2000 --which vit,fwd,fv --reps 7 --check 1 --tag chr10 >> $L 2>&1 || { tail $L; exit 1; }
grep -v amdgpu.ids $L
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY GRBM_GUI_ACTIVE -d $O/prof -o lds --output-format csv -- python3 scripts/prof_sweeps.py 2 vit,fv > $O/lds.log 2>&1 || { tail $O/lds.log; exit 1; }
python scripts/pmc_summary.py $O/prof $O/pmc.json wave_ sweep_kernel 2>&1 | head -20
timeout -k 10 200 python bench.py --cpu-1core-cols 0 --host-path 0 > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 1; }
python scripts/bench_line.py $O/bench.json bench
