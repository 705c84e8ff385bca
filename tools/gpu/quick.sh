#!/bin/bash
# Quick loop: GPU parity tests (or a -k subset), then the headline bench without the Recover/CPU lines.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/pytest_quick.log 2>&1 || { echo "gpu tests failed"; tail -40 gpurun_out/pytest_quick.log; exit 1; }
tail -2 gpurun_out/pytest_quick.log
timeout -k 10 300 python -u bench.py --steps ${BENCH_STEPS:-20} --recover-rounds 0 --c5-rounds 0 --sync-rounds 0 --no-c1 --no-cpu-baseline $BENCH_FLAGS > gpurun_out/bench_quick.json 2> gpurun_out/bench_quick.err || { echo "bench failed"; tail -30 gpurun_out/bench_quick.err; exit 1; }
python3 - <<'PY'
import json
d = json.loads(open("gpurun_out/bench_quick.json").read().strip().splitlines()[-1])
print("%.0f rounds/s" % d["value"], "ms/step %.2f" % d["ms_per_step"], "fallbacks", d.get("batch_fallbacks"))
r = d["roofline"] or {}
print("roofline", r.get("kernel"), "frac %.3f" % r.get("frac", 0), "us %.0f" % r.get("kernel_avg_us", 0))
print("iso", d.get("kernel_avg_us_isolated"))
print("ovl", d.get("kernel_avg_us"))
PY
if [ -n "$C5" ]; then
  timeout -k 10 300 python -u bench.py --steps 1 --warmup 1 --recover-rounds ${C3_ROUNDS:-0} --c5-rounds 10000 --sync-rounds 0 --no-c1 --no-cpu-baseline > gpurun_out/bench_c5.json 2> gpurun_out/bench_c5.err || { echo "c5 bench failed"; tail -30 gpurun_out/bench_c5.err; exit 1; }
  python3 - <<'PY'
import json
d = json.loads(open("gpurun_out/bench_c5.json").read().strip().splitlines()[-1])
for key in ("recover", "adversarial"):
    a = d.get(key)
    if a:
        kt = sorted(a["kernel_avg_us"].items(), key=lambda x: -x[1])[:8]
        print(key, "%.0f recovers/s" % a["value"], "s/step %.3f" % a["s_per_step"], kt)
PY
fi
