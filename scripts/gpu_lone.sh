cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
export ITR_LIB=$PWD/itrails_amd/libitrails_hip_exp.so
: > gpurun_out/lone.log
for c in 9 8 10 15 17 20 21 12; do
  ITR_VIT_CFG=$c timeout -k 10 120 python scripts/vit_lone.py 18377 1 >> gpurun_out/lone.log 2>&1 || { tail -5 gpurun_out/lone.log; exit 1; }
done
timeout -k 10 120 python scripts/vit_lone.py 18377 256 >> gpurun_out/lone.log 2>&1 || exit 1
timeout -k 10 120 python scripts/vit_lone.py 18377 512 >> gpurun_out/lone.log 2>&1 || exit 1
cat gpurun_out/lone.log
