# GPU box, round 6: (unless SKIP_TESTS) every GPU test + smoke, then the bench lines named in
# LINES ("name:args;name:args", see scripts/gpu_lines.sh); outputs under gpurun_out/$TAG.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r6}
mkdir -p $O
if [ -z "$SKIP_TESTS" ]; then
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
fi
[ -n "$LINES" ] && bash scripts/gpu_lines.sh
echo done
