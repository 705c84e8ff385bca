#!/bin/bash
# GPU parity tests, then a short bench (no CPU baseline; Recover and C5 lines on); stops at the first failure
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "gpu tests failed"; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -u bench.py --no-cpu-baseline $BENCH_FLAGS > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo "bench failed"; tail -20 gpurun_out/bench.err; exit 1; }
python - <<'PY'
import json
d = json.loads(open("gpurun_out/bench.json").read().strip().splitlines()[-1])
print("%.0f rounds/s" % d["value"], "ms/step %.2f" % d["ms_per_step"], "fallbacks", d.get("batch_fallbacks"))
r = d["roofline"] or {}
print("roofline", r.get("kernel"), "frac %.3f" % r.get("frac", 0), "us %.0f" % r.get("kernel_avg_us", 0), "chip", r.get("chip"))
print("iso", d.get("kernel_avg_us_isolated"))
for k in ("recover", "adversarial"):
    x = d.get(k) or {}
    print(k, x.get("value"), x.get("s_per_step"))
PY
python -c "import json; d=json.loads(open('gpurun_out/bench.json').read().strip().splitlines()[-1]); print('sync', d.get('sync'))"
