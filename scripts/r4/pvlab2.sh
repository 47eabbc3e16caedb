# PV Viterbi lab: sweep parity tests, diagnostic counters, product timing
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r4e}
mkdir -p $O
timeout -k 10 300 env ITR_PV=1 python -u -m pytest tests/test_gpu_sweeps.py tests/test_gpu_fullsize.py -x -q -m gpu --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 200 env ITR_LIB=itrails_amd/libitrails_hip_diag.so ITR_PV=1 python scripts/pv_lab.py lone long chr10 > $O/diag.txt 2>&1 || { tail -20 $O/diag.txt; exit 1; }
cat $O/diag.txt
timeout -k 10 200 env ITR_PV=1 python scripts/pv_lab.py lone long chr10 > $O/prod.txt 2>&1 || { tail -20 $O/prod.txt; exit 1; }
cat $O/prod.txt
