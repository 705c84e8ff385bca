#!/bin/bash
# Recover check: the -m gpu tests (or a -k selection), the probe forms, then the bench's C3 / C5 lines only.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${TESTSEL:+-k "$TESTSEL"} > gpurun_out/pytest_gpu.log 2>&1 || { echo "gpu tests failed"; tail -60 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
if [ -n "$PROBE" ]; then
timeout -k 10 120 python -u tools/microbench/probe_report.py > gpurun_out/probe.json 2> gpurun_out/probe.err || { echo "probe failed"; tail -20 gpurun_out/probe.err; exit 1; }
cat gpurun_out/probe.err
fi
timeout -k 10 600 python -u bench.py --steps 3 --no-cpu-baseline --no-c1 --sync-rounds 0 $BENCH_FLAGS > gpurun_out/bench_rec.json 2> gpurun_out/bench_rec.err || { echo "bench failed"; tail -30 gpurun_out/bench_rec.err; exit 1; }
python3 - <<'PY'
import json
d = json.loads(open("gpurun_out/bench_rec.json").read().strip().splitlines()[-1])
t = json.load(open("gpurun_out/bench_tables.json"))
for k in ("recover", "adversarial"):
    v = d.get(k) or {}
    print(k, v.get("value"), v.get("s_per_step"), v.get("roofline"))
    print("  kernels", {a: b for a, b in sorted((t.get(k) or {}).get("kernel_avg_us", {}).items(), key=lambda x: -x[1])[:12]})
PY
