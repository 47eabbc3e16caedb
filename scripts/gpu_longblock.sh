# long-block variant: 10 Mbp as 100 blocks of 100 kbp (forward + Viterbi, posterior)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --block-len 100000 --steps 5 --warmup 2 --verify 1 --host-path 0 --cpu-1core-cols 0 > gpurun_out/bench_long_fv.json 2> gpurun_out/bench_long.err || { tail -20 gpurun_out/bench_long.err; exit 1; }
timeout -k 10 300 python bench.py --block-len 100000 --mode posterior --steps 3 --warmup 1 --verify 1 --host-path 0 --cpu-1core-cols 0 > gpurun_out/bench_long_post.json 2>> gpurun_out/bench_long.err || { tail -20 gpurun_out/bench_long.err; exit 1; }
timeout -k 10 300 python bench.py --mode optimize --steps 10 --warmup 2 --verify 0 --host-path 0 --cpu-1core-cols 0 > gpurun_out/bench_opt.json 2>> gpurun_out/bench_long.err || { tail -20 gpurun_out/bench_long.err; exit 1; }
python - <<'PY'
import json
for f in ("bench_long_fv", "bench_long_post", "bench_opt"):
    d = json.load(open(f"gpurun_out/{f}.json"))
    r = d["roofline"]
    print(f, d["value"], d["unit"], "fwd", r.get("forward_ms"), "vit", r.get("viterbi_ms"), "tb", r.get("traceback_ms"), "build", d.get("build_ms"), "eq", d.get("viterbi_equal"), d.get("loglik_max_rel_err"), d.get("posterior_max_abs_err"))
PY
