# Round 4: per-wave Viterbi A/B — full-scan step (round 3) vs bound-pruned step: vit / fv
# bench lines and SQ counters of wave_vit_kernel in the Viterbi-only call
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r4t}; export O
mkdir -p $O
B="--cpu-1core-cols 0 --host-path 0"
for V in "" pruned; do
  L=""; [ -n "$V" ] && L=itrails_amd/libitrails_hip_$V.so; export ITR_LIB=$L
  timeout -k 10 300 python bench.py $B --mode vit > $O/vit$V.json 2> $O/vit$V.err || { tail $O/vit$V.err; exit 1; }
  python scripts/bench_line.py $O/vit$V.json "vit $V"
  timeout -k 10 300 python bench.py $B > $O/fv$V.json 2> $O/fv$V.err || { tail $O/fv$V.err; exit 1; }
  python scripts/bench_line.py $O/fv$V.json "chr10 $V"
  P="python3 bench.py --steps 2 --warmup 1 --verify 0 --mode vit $B"
  timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $O/prof_$V -o trace --output-format csv -- $P > $O/trace_$V.log 2>&1 || { tail $O/trace_$V.log; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU -d $O/prof_$V -o pmc1 --output-format csv -- $P > $O/pmc1_$V.log 2>&1 || { tail $O/pmc1_$V.log; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU_ADD_F64 SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_INSTS_SMEM GRBM_GUI_ACTIVE -d $O/prof_$V -o pmc2 --output-format csv -- $P > $O/pmc2_$V.log 2>&1 || { tail $O/pmc2_$V.log; exit 1; }
  python3 scripts/pmc_summary.py $O/prof_$V $O/summary_$V.json wave_vit_kernel > /dev/null || true
done
python3 - <<'PY'
import json, os
O = os.environ["O"]
for V in ("", "pruned"):
    try:
        d = json.load(open(f"{O}/summary_{V}.json"))
    except Exception as e:
        print(V, "no summary", e); continue
    for k, v in d.items():
        if "<9, 0>" in k or "wave_vit_kernel<9>" in k:
            c = v.get("counters", {})
            print(V, k[:60], {x: v.get(x) for x in ("avg_ns", "valu_busy", "wait_share", "inst_stall_share", "active_share")})
            print("   ", {x: round(c.get(x, 0)) for x in ("SQ_WAVES", "SQ_INSTS_VALU", "SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_WAVE_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_WAIT_INST_LDS", "SQ_ACTIVE_INST_VALU", "SQ_LDS_BANK_CONFLICT", "SQ_INSTS_SMEM")})
PY
echo done
