#!/bin/bash
# A/B bench of library builds: BENCH_LIBS="default path/a.so ..." x BENCH_MODES="sync async", no tests
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for lib in ${BENCH_LIBS:-default}; do
for mode in ${BENCH_MODES:-sync}; do
if [ "$lib" != default ]; then export DRAND_GPU_LIB=$GRAFT_REPO_ROOT/$lib; else unset DRAND_GPU_LIB; fi
flag=""; [ "$mode" = sync ] && flag="--sync"
timeout -k 10 300 python -u bench.py --no-cpu-baseline --recover-rounds 0 --c5-rounds 0 --steps ${BENCH_STEPS:-6} $flag $BENCH_FLAGS > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo "bench failed"; tail -20 gpurun_out/bench.err; exit 1; }
LIBNAME=$lib MODE=$mode python - <<'PY'
import json, os
d = json.loads(open("gpurun_out/bench.json").read().strip().splitlines()[-1])
print(os.environ["LIBNAME"], os.environ["MODE"], "%.0f rounds/s" % d["value"], "ms/step %.1f" % d["ms_per_step"], "fallbacks", d.get("batch_fallbacks"))
print("   ", {k: round(v) for k, v in d["kernel_avg_us"].items() if v > 300}) if d["kernel_avg_us"] else None
PY
done
done
