# Same-box A/B of environment settings on one library: for REPS rounds, each setting in
# SETTINGS ("name=VAR=val,VAR=val;name2=..."; empty assignment list = defaults) runs
# `bench.py $BENCH_ARGS` with the library $LIB (default: the product library); one line per
# run into gpurun_out/$TAG/ab.txt.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-envab}
mkdir -p $O
REPS=${REPS:-3}
B="python bench.py --verify 0 --cpu-1core-cols 0 --host-path 0 $BENCH_ARGS"
IFS=';' read -ra S <<< "$SETTINGS"
for r in $(seq $REPS); do
  for item in "${S[@]}"; do
    name=${item%%=*}; assigns=${item#*=}
    envs=(); IFS=',' read -ra A <<< "$assigns"; for x in "${A[@]}"; do [ -n "$x" ] && envs+=("$x"); done
    env ${LIB:+ITR_LIB=$PWD/$LIB} "${envs[@]}" timeout -k 10 300 $B > $O/run.json 2> $O/run.err || { tail $O/run.err; exit 1; }
    python - "$name" "$BENCH_ARGS" $O/run.json >> $O/ab.txt <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[3]) if l.startswith("{")][-1])
r = d["roofline"]
print(f"{sys.argv[1]:12s} [{sys.argv[2]}] {d['ms_per_step']:8.3f} ms/step  value {d['value']/1e6:8.1f} M  kernel {r.get('kernel_ms')}  fwd {r.get('forward_ms')}  vit {r.get('viterbi_ms')}")
PY
    tail -1 $O/ab.txt
  done
done
