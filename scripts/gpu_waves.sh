# per-wave step breakdown of the Viterbi/forward sweeps (diag build), one line per wave
cd $GRAFT_REPO_ROOT
python -c "from itrails_amd.build import build; build(force=True, diag=True)" > gpurun_out/build.log 2>&1 || exit 1
for wv in ${WAVES:-0 1 4 8}; do
  ITR_DIAG_WAVE=$wv timeout -k 10 200 python scripts/diag_probe.py 2>/dev/null | grep "1x20000" || exit 1
done
