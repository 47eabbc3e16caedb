# GPU box: every GPU test + smoke (the posterior's forward-store VALU tasks on lane groups
# inside the hybrid launch), then the (5,5) posterior A/B: product library vs a build with
# -DITR_NO_FWD_STORE_GROUPS (the VALU sweep's task), three rounds.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${TAG:-r6i}
TAG=$T SKIP_TESTS=$SKIP_TESTS LINES= bash scripts/gpu_r6.sh || exit 1
O=gpurun_out/$T
B="python bench.py --verify 0 --cpu-1core-cols 0 --host-path 0 --mode posterior --steps 5"
for r in 1 2 3; do
  for L in prod itrails_amd/libitrails_hip_nofsg.so; do
    if [ "$L" = prod ]; then LP=""; else LP="$PWD/$L"; fi
    ITR_LIB=$LP timeout -k 10 300 $B > $O/run.json 2> $O/run.err || { tail $O/run.err; exit 1; }
    python - "$L" $O/run.json >> $O/ab.txt <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[2]) if l.startswith("{")][-1])
r = d["roofline"]
print(f"{sys.argv[1]:40s} {d['ms_per_step']:8.3f} ms/step  fwd {r.get('forward_ms')}  value {d['value']/1e6:8.1f} M")
PY
    tail -1 $O/ab.txt
  done
done
echo done
