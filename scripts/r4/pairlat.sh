# Round 4: the 9-wave Viterbi step latency with 1 / 2 / 3 blocks sharing a CU: k x 8 blocks of
# 18,377 columns on the 8 reserved CUs of the Viterbi-only call (ITR_VIT_RESERVE=1 -> one CU
# per XCC, no forward set), ITR_LONG_PER_CU = k (experiment library)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r4pl2}
mkdir -p $O
export ITR_LIB=itrails_amd/libitrails_hip_exp.so ITR_VIT_RESERVE=1 ITR_FWD_RESERVE=0
for K in 1 2 3; do
  ITR_LONG_PER_CU=$K timeout -k 10 120 python scripts/vit_lone.py 18377 $((8 * K)) > $O/lat_$K.log 2>&1 || { tail $O/lat_$K.log; exit 1; }
  echo "blocks per CU $K: $(grep cfg $O/lat_$K.log)"
done
echo done
