# GPU box: build, GPU tests, forward+Viterbi bench (N=70) and posterior bench (N=133)
cd $GRAFT_REPO_ROOT
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || { echo BUILD FAIL; tail -20 gpurun_out/build.log; exit 1; }
timeout -k 10 900 python -m pytest tests -x -q -m gpu --timeout=300 --timeout-method=thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 300 python bench.py --cpu-sample 0 > gpurun_out/b_fv.json 2> gpurun_out/b_fv.err || { tail gpurun_out/b_fv.err; exit 1; }
timeout -k 10 300 python bench.py --mode posterior --n-int 7 --cpu-sample 0 > gpurun_out/b_post.json 2> gpurun_out/b_post.err || { tail gpurun_out/b_post.err; exit 1; }
python - <<'PY'
import json
for f in ("gpurun_out/b_fv.json", "gpurun_out/b_post.json"):
    d = json.load(open(f)); r = d["roofline"]
    print(f, round(d["value"] / 1e6, 1), "Mcol/s", "kernel", r["kernel_ms"], "fwd", r["forward_ms"], "frac", r["frac"])
PY
