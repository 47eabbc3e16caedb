# GPU box: a self-launched two-rank bench on the one GPU (gloo exchange), the default path.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python bench.py --gpus 2 --backend gloo --steps 3 --warmup 1 --cpu-1core-cols 0 > gpurun_out/b2.json 2> gpurun_out/b2.err || { tail -20 gpurun_out/b2.err; exit 1; }
tail -1 gpurun_out/b2.json > gpurun_out/b2l.json  # gloo prints to stdout
python scripts/bench_line.py gpurun_out/b2l.json two_ranks_one_gpu
python -c "import json; d=json.load(open('gpurun_out/b2l.json')); print(d['n_gpus'], d['config']['world_size_seen'], d['config']['parallelism'])"
