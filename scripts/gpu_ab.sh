# Same-box A/B of library builds on one bench command: for REPS rounds, each library in
# LIBS (paths relative to the repo; "prod" = the product library) runs
# `bench.py $BENCH_ARGS` once; one JSON line per run into gpurun_out/$TAG/ab.txt.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${TAG:-ab}
O=gpurun_out/$T
mkdir -p $O
REPS=${REPS:-3}
B="python bench.py --verify 0 --cpu-1core-cols 0 --host-path 0 $BENCH_ARGS"
for r in $(seq $REPS); do
  for L in $LIBS; do
    if [ "$L" = prod ]; then LP=""; else LP="$PWD/$L"; fi
    ITR_LIB=$LP timeout -k 10 300 $B > $O/run.json 2> $O/run.err || { tail $O/run.err; exit 1; }
    python - "$L" $O/run.json >> $O/ab.txt <<'PY'
import json, sys
d = json.load(open(sys.argv[2]))
r = d["roofline"]
print(f"{sys.argv[1]:40s} {d['ms_per_step']:8.3f} ms/step  value {d['value']/1e6:8.1f} M  kernel {r.get('kernel_ms')}  fwd {r.get('forward_ms')}  vit {r.get('viterbi_ms')}")
PY
    tail -1 $O/ab.txt
  done
done
