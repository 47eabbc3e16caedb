# GPU box: the other bench workloads on the current tree (config 4 base, config 3, config 5, long blocks).
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python bench.py --workload chr100 --steps 3 --warmup 1 --cpu-1core-cols 0 --host-path 0 > gpurun_out/m_chr100.json 2> gpurun_out/m.err || { tail gpurun_out/m.err; exit 1; }
python scripts/bench_line.py gpurun_out/m_chr100.json chr100
timeout -k 10 300 python bench.py --mode posterior --n-int 7 --steps 3 --warmup 1 --cpu-1core-cols 0 --host-path 0 > gpurun_out/m_post77.json 2> gpurun_out/m.err || { tail gpurun_out/m.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/m_post77.json')); print('post77', d['value'], d['ms_per_step'])"
timeout -k 10 300 python bench.py --mode optimize --steps 5 --warmup 2 --cpu-1core-cols 0 --host-path 0 > gpurun_out/m_opt55.json 2> gpurun_out/m.err || { tail gpurun_out/m.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/m_opt55.json')); print('opt55', d['value'], d['ms_per_step'])"
timeout -k 10 300 python bench.py --block-len 100000 --steps 3 --warmup 1 --cpu-1core-cols 0 --host-path 0 > gpurun_out/m_lb.json 2> gpurun_out/m.err || { tail gpurun_out/m.err; exit 1; }
python scripts/bench_line.py gpurun_out/m_lb.json longblock
