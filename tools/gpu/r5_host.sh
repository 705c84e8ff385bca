#!/bin/bash
# Round-5: where the headline's queue idle time comes from (host enqueue rate vs waits), and the C5 Recover
# kernels after the k_rs_sac table layout change (tests first).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests/ -m gpu -x -v --timeout 300 --timeout-method thread \
    -k "recover" > gpurun_out/host_pytest.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/host_pytest.log; exit 1; }
  tail -3 gpurun_out/host_pytest.log
fi
DG_BENCH_HOSTPROF=1 timeout -k 10 300 python -u bench.py --steps 20 --recover-rounds 0 --c5-rounds 0 --sync-rounds 0 \
  --no-c1 --no-cpu-baseline --no-peak-detail --no-vp-negative --neg-steps 0 > gpurun_out/host_bench.json \
  2> gpurun_out/host_bench.err || { echo "bench failed"; tail -20 gpurun_out/host_bench.err; exit 1; }
grep hostprof gpurun_out/host_bench.err
python3 -c "import json; d=json.loads(open('gpurun_out/host_bench.json').read().strip().splitlines()[-1]); print('head', d['value'], d['ms_per_step'])"
timeout -k 10 300 rocprofv3 --hip-trace --kernel-trace --output-format csv -d gpurun_out/host_trace -o run -- \
  python3 -u bench.py --steps 10 --recover-rounds 0 --c5-rounds 0 --sync-rounds 0 --no-c1 --no-cpu-baseline \
  --no-peak-detail --no-vp-negative --neg-steps 0 --no-kernel-timing > gpurun_out/host_trace.json \
  2> gpurun_out/host_trace.err || { echo "hip trace failed"; tail -20 gpurun_out/host_trace.err; exit 1; }
if [ -z "$SKIP_C5" ]; then
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c5_prof -o run -- \
    python3 -u bench.py --steps 3 --recover-rounds 0 --sync-rounds 0 --no-c1 --no-cpu-baseline --no-peak-detail \
    --no-vp-negative --neg-steps 0 > gpurun_out/c5.json 2> gpurun_out/c5.err \
    || { echo "c5 failed"; tail -20 gpurun_out/c5.err; exit 1; }
  grep -E '"k_rs_sac"|"k_ck_miller"|"k_rs_tab_add"' gpurun_out/c5_prof/run_kernel_stats.csv
  python3 -c "import json; d=json.loads(open('gpurun_out/c5.json').read().strip().splitlines()[-1]); a=d.get('adversarial') or {}; print('c5', a.get('value'), a.get('unit'))"
fi
if [ -n "$NEG_TRACE" ]; then
  DG_XR_SKIP=${DG_XR_SKIP:-1} timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/neg_trace \
    -o run -- python3 -u bench.py --steps 3 --recover-rounds 0 --c5-rounds 0 --sync-rounds 0 --no-c1 \
    --no-cpu-baseline --no-peak-detail --no-vp-negative --neg-steps 5 --no-kernel-timing > gpurun_out/neg_trace.json \
    2> gpurun_out/neg_trace.err || { echo "neg trace failed"; tail -20 gpurun_out/neg_trace.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/neg_trace.json').read().strip().splitlines()[-1]); print('neg', d['c2_negative']['value'])"
fi
