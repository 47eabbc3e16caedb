# Round 4: bound-pruned per-wave Viterbi with re-tuned long sets (the pruned step has a
# higher per-column latency and a lower per-column cost): Viterbi-only long set
# (ITR_VIT_NLONG_V) and forward+Viterbi wave latency (ITR_WAVE_LAT), experiment library
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r4v}
mkdir -p $O
B="--cpu-1core-cols 0 --host-path 0 --verify 0"
export ITR_LIB=itrails_amd/libitrails_hip_prunedexp.so
for K in 69 90 110 130 160; do
  ITR_VIT_NLONG_V=$K timeout -k 10 200 python bench.py $B --mode vit > $O/vit$K.json 2> $O/vit$K.err || { tail $O/vit$K.err; exit 1; }
  python scripts/bench_line.py $O/vit$K.json "vit nlong_v $K"
done
for W in 800e-9 1000e-9 1300e-9 1700e-9; do
  ITR_WAVE_LAT=$W timeout -k 10 200 python bench.py $B > $O/fv$W.json 2> $O/fv$W.err || { tail $O/fv$W.err; exit 1; }
  python scripts/bench_line.py $O/fv$W.json "chr10 wave_lat $W"
done
echo done
