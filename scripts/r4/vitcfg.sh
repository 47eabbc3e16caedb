# Round 4: lone-step latency of the long-block Viterbi layouts (experiment library,
# ITR_VIT_CFG = hmm_sweeps.hip kCfgs index): 100 x 100 kbp forward+Viterbi and chr10 Viterbi-only
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r4vc}
mkdir -p $O
B="--cpu-1core-cols 0 --host-path 0"
export ITR_LIB=itrails_amd/libitrails_hip_exp.so
for C in 9 15 20 2 19; do
  ITR_VIT_CFG=$C timeout -k 10 300 python bench.py $B --block-len 100000 --steps 3 > $O/lb_c$C.json 2> $O/lb_c$C.err || { tail -3 $O/lb_c$C.err; continue; }
  python scripts/bench_line.py $O/lb_c$C.json "longblock cfg $C"
done
echo done
