# Same-box A/B over (library, settings) pairs: RUNS = "label|lib|VAR=v,VAR2=w ..." items
# ("prod" = the product library), REPS rounds, one line per run into gpurun_out/$TAG/ab.txt
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-abenv}
mkdir -p $O
for r in $(seq ${REPS:-2}); do
  for item in $RUNS; do
    IFS='|' read lab lib envs <<< "$item"
    if [ "$lib" = prod ]; then LP=""; else LP="$PWD/$lib"; fi
    env ITR_LIB=$LP ${envs//,/ } timeout -k 10 300 python bench.py --verify 0 --cpu-1core-cols 0 --host-path 0 $BENCH_ARGS > $O/run.json 2> $O/run.err || { tail $O/run.err; exit 1; }
    python - "$lab" $O/run.json >> $O/ab.txt <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[2]) if l.startswith("{")][-1])
r = d["roofline"]
print(f"{sys.argv[1]:16s} {d['ms_per_step']:8.3f} ms/step  value {d['value']/1e6:8.1f} M  kernel {r.get('kernel_ms')}  fwd {r.get('forward_ms')}")
PY
  done
done
cat $O/ab.txt
