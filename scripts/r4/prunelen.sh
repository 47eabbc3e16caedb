# Round 4: per-wave Viterbi with both steps in one kernel — blocks shorter than ITR_PRUNE_LEN
# take the bound-pruned step, the others the full scan (experiment library).  Parity first
# (all pruned / mixed, against the CPU restatement), then the threshold sweep on chr10
# (Viterbi-only and forward+Viterbi) and chr100.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r4pl}
mkdir -p $O
B="--cpu-1core-cols 0 --host-path 0 --verify 0"
export ITR_LIB=itrails_amd/libitrails_hip_exp.so
for L in 1000000 1000; do
  ITR_PRUNE_LEN=$L timeout -k 10 300 python scripts/kernel_lab.py --which vit,fv --check 1 --tag "prune<$L" > $O/check_$L.log 2>&1 || { tail $O/check_$L.log; exit 1; }
  cat $O/check_$L.log
done
for L in ${LENS:-0 400 800 1200 1600 2400 1000000}; do
  ITR_PRUNE_LEN=$L timeout -k 10 300 python bench.py $B --mode vit > $O/vit_$L.json 2> $O/vit_$L.err || { tail $O/vit_$L.err; exit 1; }
  python scripts/bench_line.py $O/vit_$L.json "vit prune<$L"
  ITR_PRUNE_LEN=$L timeout -k 10 300 python bench.py $B > $O/fv_$L.json 2> $O/fv_$L.err || { tail $O/fv_$L.err; exit 1; }
  python scripts/bench_line.py $O/fv_$L.json "chr10 prune<$L"
done
for L in 0 ${C100:-1200 1000000}; do
  ITR_PRUNE_LEN=$L timeout -k 10 300 python bench.py $B --workload chr100 --steps 3 --warmup 1 > $O/c100_$L.json 2> $O/c100_$L.err || { tail $O/c100_$L.err; exit 1; }
  python scripts/bench_line.py $O/c100_$L.json "chr100 prune<$L"
done
echo done
