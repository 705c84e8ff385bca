#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/bench_call1.json 2> gpurun_out/bench_call1.err || { echo "bench1 failed"; tail -20 gpurun_out/bench_call1.err; exit 1; }
DRAND_GPU_LIB=$GRAFT_REPO_ROOT/drand_amd/libdrandgpu_call0.so timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/bench_call0.json 2> gpurun_out/bench_call0.err || { echo "bench0 failed"; tail -20 gpurun_out/bench_call0.err; exit 1; }
python - <<'PY'
import json
for f in ("gpurun_out/bench_call1.json", "gpurun_out/bench_call0.json"):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f, "%.0f rounds/s" % d["value"], "ms/step %.1f" % d["ms_per_step"], d["kernel_avg_us"])
PY
