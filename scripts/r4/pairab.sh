# Round 4: same-box A/B of the paired long set: product plan (kVitPair 407 ns), the plan with
# a 360 ns paired step (fewer reserved CUs), and one long block per reserved CU; chr10
# forward+Viterbi, default bench (10 warmup, 20 steps), interleaved (experiment library)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r4pab}
mkdir -p $O
B="--cpu-1core-cols 0 --host-path 0 --verify 0"
export ITR_LIB=itrails_amd/libitrails_hip_exp.so
for i in ${RUNS:-1 2 3}; do
  for L in ${VARS:-paired 360 1}; do
    unset ITR_LONG_PER_CU ITR_VIT_PAIR; [ $L = 1 ] && export ITR_LONG_PER_CU=1; [ $L = 360 ] && export ITR_VIT_PAIR=360e-9
    timeout -k 10 300 python bench.py $B > $O/fv_$L.$i.json 2> $O/fv_$L.$i.err || { tail $O/fv_$L.$i.err; exit 1; }
    python scripts/bench_line.py $O/fv_$L.$i.json "chr10 long set $L run $i"
  done
done
echo done
