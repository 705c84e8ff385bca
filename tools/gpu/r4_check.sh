#!/bin/bash
# Round-4 check: every -m gpu test (the 1M-chain shard test included), then the full default bench; stops at the
# first failure.  SKIP_TESTS=1 / SKIP_BENCH=1 skip a part; PYTEST_K selects tests; BENCH_FLAGS adds bench options.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
if [ -z "$SKIP_TESTS" ]; then
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/pytest_gpu.log 2>&1 || { echo "gpu tests failed"; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
fi
if [ -z "$SKIP_BENCH" ]; then
timeout -k 10 800 python -u bench.py --steps ${BENCH_STEPS:-20} $BENCH_FLAGS > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo "bench failed"; tail -30 gpurun_out/bench.err; exit 1; }
wc -c gpurun_out/bench.json
tail -c 5000 gpurun_out/bench.json
fi
