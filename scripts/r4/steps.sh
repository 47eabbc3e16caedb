# Round 4: step-time spread of the default forward+Viterbi bench (20 timed steps, twice, plus
# the default 5-step run)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r4st}
mkdir -p $O
B="--cpu-1core-cols 0 --host-path 0 --verify 0"
for i in 1 2; do
  timeout -k 10 300 python bench.py $B --steps 20 --warmup 3 > $O/s20_$i.json 2> $O/s20_$i.err || { tail $O/s20_$i.err; exit 1; }
  python scripts/bench_line.py $O/s20_$i.json "chr10 20 steps run $i"
done
timeout -k 10 300 python bench.py $B > $O/s5.json 2> $O/s5.err || { tail $O/s5.err; exit 1; }
python scripts/bench_line.py $O/s5.json "chr10 5 steps"
echo done
