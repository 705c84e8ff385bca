#!/bin/bash
# Round-5 check: the round-5 GPU tests first, then every -m gpu test, then the negative bench lines (BENCH_FLAGS adds
# options).  Stops at the first failure.  SKIP_TESTS=1 / SKIP_ALL=1 / SKIP_BENCH=1 skip parts; PYTEST_K selects.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
if [ -z "$SKIP_TESTS" ]; then
timeout -k 10 600 python -u -m pytest tests/test_gpu_round5.py -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/pytest_r5.log 2>&1 || { echo "r5 gpu tests failed"; tail -60 gpurun_out/pytest_r5.log; exit 1; }
tail -3 gpurun_out/pytest_r5.log
fi
if [ -z "$SKIP_ALL" ]; then
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "gpu tests failed"; tail -60 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
fi
if [ -z "$SKIP_BENCH" ]; then
timeout -k 10 900 python -u bench.py --steps ${BENCH_STEPS:-10} --recover-rounds 0 --sync-rounds 0 --no-c1 \
  --no-cpu-baseline --neg-steps ${NEG_STEPS:-10} --tables-out gpurun_out/neg_tables.json $BENCH_FLAGS \
  > gpurun_out/neg.json 2> gpurun_out/neg.err || { echo "bench failed"; tail -30 gpurun_out/neg.err; exit 1; }
tail -c 6000 gpurun_out/neg.json
fi
