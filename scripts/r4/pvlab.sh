# PV Viterbi lab: diagnostic library counters on lone / long / chr10, then the product timing
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r4c}
mkdir -p $O
timeout -k 10 200 env ITR_LIB=itrails_amd/libitrails_hip_diag.so python scripts/pv_lab.py lone long chr10 > $O/diag.txt 2>&1 || { tail -20 $O/diag.txt; exit 1; }
cat $O/diag.txt
timeout -k 10 200 python scripts/pv_lab.py lone long chr10 > $O/prod.txt 2>&1 || { tail -20 $O/prod.txt; exit 1; }
cat $O/prod.txt
