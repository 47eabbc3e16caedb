# posterior parity tests on the product library, then a same-box A/B of library builds on the
# (7,7) posterior: all-matrix-core uniform blocks, then the default workload
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r5pab}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu -k "post or 133 or 77" --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
ITR_POST_URGENT_FRAC=1.01 TAG=$TAG/u REPS=2 LIBS="$LIBS" BENCH_ARGS="--mode posterior --n-int 7 --steps 3 --warmup 1 --block-len 2000" bash scripts/gpu_ab.sh || exit 1
cat $O/u/ab.txt
TAG=$TAG/d REPS=2 LIBS="$LIBS" BENCH_ARGS="--mode posterior --n-int 7 --steps 3 --warmup 1" bash scripts/gpu_ab.sh || exit 1
cat $O/d/ab.txt
