#!/bin/bash
# A/B bench of two library builds (BENCH_LIB_B), no tests
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for lib in "" "$BENCH_LIB_B"; do
if [ -n "$lib" ]; then export DRAND_GPU_LIB=$GRAFT_REPO_ROOT/$lib; fi
timeout -k 10 300 python -u bench.py --no-cpu-baseline --recover-rounds 0 --steps 6 > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo "bench failed"; tail -20 gpurun_out/bench.err; exit 1; }
python - <<'PY'
import json, os
d = json.loads(open("gpurun_out/bench.json").read().strip().splitlines()[-1])
print(os.environ.get("DRAND_GPU_LIB", "default"), "%.0f rounds/s" % d["value"], "ms/step %.1f" % d["ms_per_step"])
print({k: round(v) for k, v in d["kernel_avg_us"].items() if v > 500}, "fallbacks", d.get("batch_fallbacks"))
PY
done
