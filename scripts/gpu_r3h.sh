# Round 3: long-block forward+Viterbi (one CU per block beside the forward) with its check;
# posterior (7,7) lab: one-block latencies and the VALU/matrix-core split
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r3h
mkdir -p $O
timeout -k 10 400 python bench.py --block-len 100000 --mbp 10 --cpu-1core-cols 0 --host-path 0 --steps 5 > $O/longblock.json 2> $O/longblock.err || { tail $O/longblock.err; exit 1; }
python scripts/bench_line.py $O/longblock.json longblock
for L in 20000 5000; do
timeout -k 10 200 python bench.py --mode posterior --n-int 7 --block-len $L --mbp $(python -c "print($L/1e6)") --cpu-1core-cols 0 --host-path 0 --verify 0 --steps 3 > $O/post1_$L.json 2> $O/post1_$L.err || { tail $O/post1_$L.err; exit 1; }
python scripts/bench_line.py $O/post1_$L.json post_one_block_$L
done
for F in 0.3 0.7 2.0; do
timeout -k 10 200 env ITR_LIB=itrails_amd/libitrails_hip_exp.so ITR_POST_URGENT_FRAC=$F python bench.py --mode posterior --n-int 7 --cpu-1core-cols 0 --host-path 0 --verify 0 --steps 3 > $O/post_pf$F.json 2> $O/post_pf$F.err || { tail $O/post_pf$F.err; exit 1; }
python scripts/bench_line.py $O/post_pf$F.json post_pfrac_$F
done
