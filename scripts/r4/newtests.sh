# Round 4: new GPU tests (few-block branch, every chr100 shard, device-built model decode)
# and the chr100 shard projection
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r4n}; export O
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_sweeps.py tests/test_gpu_fullsize.py -x -v -s -m gpu --timeout 300 --timeout-method thread -k "few_long or chr100_shard or device_built" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
grep -E "PASSED|FAILED|viterbi_columns_differing" $O/pytest.log | tail -20
timeout -k 10 400 python bench.py --workload chr100 --steps 3 --cpu-1core-cols 0 --host-path 0 --verify 0 --project-shards 8 > $O/chr100.json 2> $O/chr100.err || { tail $O/chr100.err; exit 1; }
python - <<'PY'
import json, os
d = json.load(open(os.environ.get("O", "gpurun_out/r4n") + "/chr100.json"))
print(d["value"], d["ms_per_step"], json.dumps(d["shard_projection"]))
PY
