#!/bin/bash
# tests + pipelined bench + sync bench (no CPU baseline, no recover); stops at the first failure
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
for mode in "" "--async"; do
timeout -k 10 300 python -u bench.py --no-cpu-baseline --recover-rounds 0 --steps 6 $mode ${BENCH_ARGS} > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo "bench failed"; tail -20 gpurun_out/bench.err; exit 1; }
python - <<'PY'
import json
d = json.loads(open("gpurun_out/bench.json").read().strip().splitlines()[-1])
print("%.0f rounds/s" % d["value"], "ms/step %.1f" % d["ms_per_step"], "roof", d["roofline"] and round(d["roofline"]["frac"], 4), d["roofline"] and d["roofline"]["kernel"])
print({k: round(v) for k, v in d["kernel_avg_us"].items()})
PY
done
