cd $GRAFT_REPO_ROOT
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || exit 1
for c in "4 fwd short" "1 fwd short" "4 fwd noempty" "4 fwd all" "1 fwd all" "1 vit all" "1 post all" "4 vit all" "4 post all"; do
  echo "== $c" | tee -a gpurun_out/debug.log
  timeout -k 5 60 python scripts/debug_case.py $c >> gpurun_out/debug.log 2>&1
  rc=$?
  echo "rc=$rc" | tee -a gpurun_out/debug.log
  if [ $rc -ne 0 ]; then exit $rc; fi
done
