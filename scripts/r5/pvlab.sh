cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r5h}
mkdir -p $O
ITR_LIB=$PWD/itrails_amd/libitrails_hip_exp.so timeout -k 10 600 python scripts/pv_lab.py > $O/pv_lab.txt 2>&1 || { tail -20 $O/pv_lab.txt; exit 1; }
cat $O/pv_lab.txt
