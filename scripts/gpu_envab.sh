# Same-box A/B of environment settings on one bench command with one library ($LIB, default
# the experiment build): for REPS rounds, each setting in $SETS ("label:VAR=v,VAR2=w" items,
# "base:" = none) runs `bench.py $BENCH_ARGS`; one line per run into gpurun_out/$TAG/envab.txt
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-envab}
mkdir -p $O
LIBP=$PWD/${LIB:-itrails_amd/libitrails_hip_exp.so}
for r in $(seq ${REPS:-2}); do
  for S in $SETS; do
    label=${S%%:*}; vars=${S#*:}
    envs=$(echo "$vars" | tr ',' ' ')
    env ITR_LIB=$LIBP $envs timeout -k 10 300 python bench.py --cpu-1core-cols 0 --host-path 0 $BENCH_ARGS > $O/run.json 2> $O/run.err || { tail $O/run.err; exit 1; }
    python - "$label" $O/run.json >> $O/envab.txt <<'PY'
import json, sys
d = json.load(open(sys.argv[2]))
r = d["roofline"]
print(f"{sys.argv[1]:24s} {d['ms_per_step']:8.3f} ms/step  {d['value']/1e6:8.1f} M  kernel {r.get('kernel_ms')}  vit_eq {d.get('viterbi_equal')}")
PY
    tail -1 $O/envab.txt
  done
done
