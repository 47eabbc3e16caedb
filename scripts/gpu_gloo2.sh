# Rehearse the multi-rank bench on the one-GPU box: two ranks on cuda:0, the per-block
# log-likelihood exchange over gloo (the driver's N > 1 runs use RCCL over xGMI).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 1 \
  --backend gloo --cpu-sample 0 > gpurun_out/bench_gloo2.json 2> gpurun_out/bench_gloo2.err
rc=$?
cat gpurun_out/bench_gloo2.json
tail -3 gpurun_out/bench_gloo2.err
exit $rc
