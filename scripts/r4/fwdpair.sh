# Round 4: two forward VALU halves per reserved CU at a time (ITR_FWD_PER_CU) with fewer
# forward CUs (ITR_FWD_RESERVE, before the 8-CU rounding; product: 20 -> 24), chr10
# forward+Viterbi default bench twice per variant (experiment library of the lab's tree: the
# ITR_FWD_PER_CU knob is not in the committed tree)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r4fp}
mkdir -p $O
B="--cpu-1core-cols 0 --host-path 0 --verify 0"
export ITR_LIB=itrails_amd/libitrails_hip_exp.so
for V in ${VARS:-1:0 2:16 2:10 2:8 1:0}; do
  IFS=: read FP FR <<< "$V"
  unset ITR_FWD_PER_CU ITR_FWD_RESERVE
  [ $FP != 1 ] && export ITR_FWD_PER_CU=$FP
  [ $FR != 0 ] && export ITR_FWD_RESERVE=$FR
  for i in 1 2; do
    timeout -k 10 300 python bench.py $B > $O/fv_$V.$i.json 2> $O/fv_$V.$i.err || { tail $O/fv_$V.$i.err; exit 1; }
    python scripts/bench_line.py $O/fv_$V.$i.json "chr10 fwd per_cu:reserve $V run $i"
  done
done
echo done
