"""Print one summary line of a bench.py JSON result (experiment scripts)."""
import json
import sys

# the last JSON line (RCCL may print its version banner on stdout first)
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
r = d["roofline"]
print(" ".join(sys.argv[2:]), round(d["value"] / 1e6, 1), "Mcol/s fwd", r.get("forward_ms"),
      "vit", r.get("kernel_ms"), "trace", r.get("traceback_ms"), "fv", r.get("forward_viterbi_ms"),
      "ms/step", d.get("ms_per_step"), "vit_eq", d.get("viterbi_equal"), "ll_err", d.get("loglik_max_rel_err"))
extra = {k: d[k] for k in ("posterior_allclose_1e-8", "posterior_max_rel_err", "build_ms",
                           "per_rank_step_ms", "allreduce_ms") if k in d}
if extra:
    print("   ", extra, "traffic", r.get("traffic"))
