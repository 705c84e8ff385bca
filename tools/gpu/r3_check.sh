#!/bin/bash
# Round-3 check: every -m gpu test, the peak-probe forms, then the full default bench; stops at the first failure.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
if [ -z "$SKIP_TESTS" ]; then
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "gpu tests failed"; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
fi
timeout -k 10 120 python -u tools/microbench/probe_report.py > gpurun_out/probe.json 2> gpurun_out/probe.err || { echo "probe failed"; tail -20 gpurun_out/probe.err; exit 1; }
cat gpurun_out/probe.err
timeout -k 10 700 python -u bench.py --steps ${BENCH_STEPS:-20} $BENCH_FLAGS > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo "bench failed"; tail -30 gpurun_out/bench.err; exit 1; }
wc -c gpurun_out/bench.json
tail -c 5000 gpurun_out/bench.json
