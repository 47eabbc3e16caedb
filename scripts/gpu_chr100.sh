# GPU box: chr100 (config 4 base) with the forward split even when its VALU halves outnumber
# the reserved CUs (experiment knob), then the default chr10 bench.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
ITR_LIB=itrails_amd/libitrails_hip_exp.so ITR_FV_SPLIT_CAP=100000 timeout -k 10 400 python bench.py --workload chr100 --steps 3 --warmup 1 --verify 0 --cpu-1core-cols 0 --host-path 0 > gpurun_out/m_chr100b.json 2> gpurun_out/m.err || { tail gpurun_out/m.err; exit 1; }
python scripts/bench_line.py gpurun_out/m_chr100b.json chr100_split_all
timeout -k 10 200 python bench.py --cpu-1core-cols 0 --host-path 0 > gpurun_out/m_chr10b.json 2> gpurun_out/m.err || { tail gpurun_out/m.err; exit 1; }
python scripts/bench_line.py gpurun_out/m_chr10b.json chr10
