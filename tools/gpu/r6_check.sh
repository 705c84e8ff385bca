#!/bin/bash
# Round-6 check: the round-5/6 GPU tests first, then every -m gpu test, then the driver's bench command
# (bench.py --gpus 1 --steps 20 --warmup 5) -> gpurun_out/r6_bench.json.  Stops at the first failure.
# SKIP_TESTS=1 / SKIP_ALL=1 / SKIP_BENCH=1 skip parts; PYTEST_K selects among the round-5/6 tests; BENCH_FLAGS adds options.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests/test_gpu_round5.py -m gpu -x -v -s --timeout 300 --timeout-method thread \
    ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/r6_pytest_r5.log 2>&1 || { echo "r5 gpu tests failed"; tail -60 gpurun_out/r6_pytest_r5.log; exit 1; }
  tail -3 gpurun_out/r6_pytest_r5.log
fi
if [ -z "$SKIP_ALL" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    > gpurun_out/r6_pytest_gpu.log 2>&1 || { echo "gpu tests failed"; tail -60 gpurun_out/r6_pytest_gpu.log; exit 1; }
  tail -3 gpurun_out/r6_pytest_gpu.log
fi
if [ -z "$SKIP_BENCH" ]; then
  timeout -k 10 900 python -u bench.py --gpus 1 --steps 20 --warmup 5 $BENCH_FLAGS > gpurun_out/r6_bench.json \
    2> gpurun_out/r6_bench.err || { echo "bench failed"; tail -30 gpurun_out/r6_bench.err; exit 1; }
  python3 - <<'PY'
import json
d = json.loads(open("gpurun_out/r6_bench.json").read().strip().splitlines()[-1])
print("head", d["value"], d["ms_per_step"], "roof", d["roofline"].get("frac"))
for k in ("recover", "c2_verify_all", "adversarial", "c1", "c2_negative", "vp_negative", "sync", "live_latency"):
    v = d.get(k) or {}
    print(k, v.get("value"), v.get("unit"), {a: b for a, b in v.items() if a.endswith("_ms")} if k == "live_latency" else "")
PY
fi
