# Round 3: lone-step latency components (micro), then the default bench twice (variance).
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3b
timeout -k 10 60 scripts/micro/latency > gpurun_out/r3b/latency.txt 2>&1 || { cat gpurun_out/r3b/latency.txt; exit 1; }
cat gpurun_out/r3b/latency.txt
for i in 1 2; do
timeout -k 10 300 python bench.py --verify 0 --cpu-1core-cols 0 --host-path 0 --steps 10 > gpurun_out/r3b/bench$i.json 2> gpurun_out/r3b/bench$i.err || { tail gpurun_out/r3b/bench$i.err; exit 1; }
python scripts/bench_line.py gpurun_out/r3b/bench$i.json run$i
done
