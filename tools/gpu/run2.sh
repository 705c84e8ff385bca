#!/bin/bash
# full-size bench with CPU baseline, then rocprofv3 kernel stats of a short bench
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u bench.py > gpurun_out/bench_full.json 2> gpurun_out/bench_full.err || { echo "bench failed"; tail -20 gpurun_out/bench_full.err; exit 1; }
cat gpurun_out/bench_full.json
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof1" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 2 --warmup 1 --no-cpu-baseline > "$GRAFT_REPO_ROOT/gpurun_out/prof1.log" 2>&1 || { echo "rocprof failed"; tail -20 "$GRAFT_REPO_ROOT/gpurun_out/prof1.log"; exit 1; }
find "$GRAFT_REPO_ROOT/gpurun_out/prof1" -name "*stats*" | head
