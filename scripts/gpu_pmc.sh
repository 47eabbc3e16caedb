# SQ issue/wait counters for the sweep kernels (one rocprofv3 --pmc pass per counter set).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
B="python3 bench.py --steps 2 --warmup 1 --cpu-sample 0 ${BENCH_ARGS}"
TAG=${TAG:-pmc}
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_INST_LDS SQ_BUSY_CYCLES -d gpurun_out/$TAG -o sq --output-format csv -- $B > gpurun_out/${TAG}_sq.log 2>&1 || { tail gpurun_out/${TAG}_sq.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_WAVES GRBM_GUI_ACTIVE -d gpurun_out/$TAG -o lds --output-format csv -- $B > gpurun_out/${TAG}_lds.log 2>&1 || { tail gpurun_out/${TAG}_lds.log; exit 1; }
python3 - <<'PY'
import csv, glob, collections, os
tag = os.environ.get("TAG", "pmc")
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(f"gpurun_out/{tag}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        agg[r["Kernel_Name"][:48]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in agg.items():
    if "sweep" not in k and "trace" not in k: continue
    print(k, {c: round(sum(v) / len(v)) for c, v in sorted(d.items())})
PY
