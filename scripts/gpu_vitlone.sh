# GPU box: lone-block Viterbi step of the lane-group layout against the 9-wave layout (same
# experiment library, ITR_VIT_CFG), one and two blocks per CU, then the Viterbi GPU tests.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-vitlone}
mkdir -p $O
X=$PWD/itrails_amd/libitrails_hip_exp.so
for T in 18377 100000; do
  for c in 9 22; do
    ITR_LIB=$X ITR_VIT_CFG=$c timeout -k 10 120 python scripts/vit_lone.py $T 1 >> $O/lone.txt 2>&1 || { tail $O/lone.txt; exit 1; }
  done
done
for c in 9 22; do
  ITR_LIB=$X ITR_VIT_CFG=$c timeout -k 10 120 python scripts/vit_lone.py 18377 512 >> $O/lone.txt 2>&1 || { tail $O/lone.txt; exit 1; }
done
cat $O/lone.txt
timeout -k 10 900 python -u -m pytest tests/test_gpu_sweeps.py tests/test_gpu_rows.py -x -q -m gpu --timeout 300 --timeout-method thread > $O/pytest_sweeps.log 2>&1 || { tail -40 $O/pytest_sweeps.log; exit 1; }
tail -1 $O/pytest_sweeps.log
[ -n "$LINES" ] && bash scripts/gpu_lines.sh
echo done
