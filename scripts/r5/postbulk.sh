# (7,7) posterior: bulk-only workload (uniform 2000-column blocks) against the default one,
# and the share of long blocks on VALU tasks (experiment build)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r5pb}
mkdir -p $O
B="--cpu-1core-cols 0 --host-path 0 --verify 0 --mode posterior --n-int 7 --steps 3 --warmup 1"
for cfg in ${CFGS:-"uniform2000:--block-len 2000:" "default::"}; do
  IFS=: read lab args envs <<< "$cfg"; args=${args//@/ }; envs=${envs//@/ }
  env ITR_LIB=$PWD/itrails_amd/libitrails_hip_exp.so $envs timeout -k 10 300 python bench.py $B $args > $O/$lab.json 2> $O/$lab.err || { tail $O/$lab.err; exit 1; }
  python scripts/bench_line.py $O/$lab.json $lab
done
echo done
