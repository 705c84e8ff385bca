#!/bin/bash
# kernel trace of the asynchronous bench (timeline of overlapping batches)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out/trace
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/trace -o run -- python3 $R/bench.py --steps 8 --warmup 1 --no-cpu-baseline --recover-rounds 0 --c5-rounds 0 --no-kernel-timing ${TRACE_FLAGS:-} > $R/gpurun_out/trace/log.txt 2>&1 || { echo "trace failed"; tail -20 $R/gpurun_out/trace/log.txt; exit 1; }
find $R/gpurun_out/trace -name "*.csv"
