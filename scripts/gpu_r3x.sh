# Round 3: planned CU partition (plan_partition) + reserved CUs joining the bulk queue: parity,
# + separate reserved sets (long Viterbi / forward halves) each joining the bulk queue on its own
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r3x
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_sweeps.py tests/test_gpu_fullsize.py -x -q -m gpu --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
L=$O/lab.txt
: > $L
X=ITR_LIB=itrails_amd/libitrails_hip_exp.so
run() { timeout -k 10 150 env $X "$@" >> $L 2>&1 || { tail $L; exit 1; }; }
K="python scripts/kernel_lab.py --mean-block 2000 --which fv --reps 9"
run env ITR_VERBOSE=1 python scripts/kernel_lab.py --mean-block 2000 --which vit,fv --reps 9 --check 1 --tag default
for i in 1 2; do
  run $K --tag "planned_$i"
  run ITR_WAVE_LAT=0.7e-6 $K --tag "wlat0.7_$i"
  run ITR_WAVE_LAT=0.9e-6 $K --tag "wlat0.9_$i"
  run ITR_FWD_RESERVE=12 $K --tag "rf12_$i"
done
run python scripts/kernel_lab.py --mean-block 2000 --mbp 100 --which vit,fv --reps 3 --check 1 --tag chr100; run env ITR_VERBOSE=1 python scripts/kernel_lab.py --mean-block 2000 --mbp 100 --which fv --reps 1 --tag chr100v
run python scripts/kernel_lab.py --mean-block 300 --which vit,fv --reps 5 --tag short300
run python scripts/kernel_lab.py --block-len 100000 --which fv --reps 3 --tag longblock
run python scripts/kernel_lab.py --mean-block 2000 --mbp 12.5 --which fv --reps 5 --check 1 --tag chr12.5
grep -v amdgpu.ids $L
