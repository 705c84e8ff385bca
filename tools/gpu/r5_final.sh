#!/bin/bash
# Round-5 full check: every GPU test, then the default bench.py run (all lines) -> profiles/r5_bench_full.json.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 1000 python -u -m pytest tests/ -m gpu -x -v --timeout 300 --timeout-method thread \
    > gpurun_out/final_pytest.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/final_pytest.log; exit 1; }
  tail -2 gpurun_out/final_pytest.log
fi
timeout -k 10 900 python -u bench.py > gpurun_out/final_bench.json 2> gpurun_out/final_bench.err \
  || { echo "bench failed"; tail -30 gpurun_out/final_bench.err; exit 1; }
python3 - <<'PY'
import json
d = json.loads(open("gpurun_out/final_bench.json").read().strip().splitlines()[-1])
print("head", d["value"], d["ms_per_step"], "roof", d["roofline"].get("frac"))
for k in ("recover", "c2_verify_all", "adversarial", "c1", "c2_negative", "vp_negative", "sync", "live_latency"):
    v = d.get(k) or {}
    print(k, v.get("value"), v.get("unit"))
print("bytes", len(open("gpurun_out/final_bench.json").read().strip().splitlines()[-1]))
PY
