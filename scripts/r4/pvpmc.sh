# PV Viterbi counters on chr10 (one pass per counter set)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r4k}; export O
mkdir -p $O
export ITR_PV=1
P="python3 scripts/pv_lab.py ${WL:-chr10}"
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $O/prof -o trace --output-format csv -- $P > $O/trace.log 2>&1 || { tail $O/trace.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU -d $O/prof -o pmc1 --output-format csv -- $P > $O/pmc1.log 2>&1 || { tail $O/pmc1.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_WAIT_ANY SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE -d $O/prof -o pmc2 --output-format csv -- $P > $O/pmc2.log 2>&1 || { tail $O/pmc2.log; exit 1; }
python3 - <<'PY'
import csv, glob, collections, os
O = os.environ.get("O", "gpurun_out/r4k")
for f in sorted(glob.glob(f"{O}/prof/**/*counter_collection.csv", recursive=True)):
    agg = collections.defaultdict(float); cnt = collections.defaultdict(int)
    for row in csv.DictReader(open(f)):
        if "pv_vit" not in row.get("Kernel_Name", ""): continue
        agg[row["Counter_Name"]] += float(row["Counter_Value"]); cnt[row["Counter_Name"]] += 1
    print(f)
    for k, v in sorted(agg.items()): print(f"  {k:28s} {v:16.0f}  (dispatch-rows {cnt[k]})")
PY
