#!/bin/bash
# GPU parity tests, then the full default bench; stops at the first failure.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "gpu tests failed"; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
timeout -k 10 700 python -u bench.py --steps ${BENCH_STEPS:-20} $BENCH_FLAGS > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo "bench failed"; tail -30 gpurun_out/bench.err; exit 1; }
python3 - <<'PY'
import json
d = json.loads(open("gpurun_out/bench.json").read().strip().splitlines()[-1])
print("%.0f rounds/s" % d["value"], "ms/step %.2f" % d["ms_per_step"], "fallbacks", d.get("batch_fallbacks"))
r = d["roofline"] or {}
print("roofline", r.get("kernel"), "frac %.3f" % r.get("frac", 0), "us %.0f" % r.get("kernel_avg_us", 0))
for k in ("recover", "adversarial", "c1", "live_latency", "sync", "cpu_baseline"):
    v = d.get(k) or {}
    print(k, {x: y for x, y in v.items() if not isinstance(y, dict) and x not in ("note", "metric")},
          (v.get("cpu_baseline") or {}).get("value"), (v.get("roofline") or {}).get("frac"))
print("iso", d.get("kernel_avg_us_isolated"))
PY
