#!/bin/bash
# GPU tests, then the C5 line alone (headline 1 step, no CPU legs); stops at the first failure.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
if [ -z "$SKIP_TESTS" ]; then
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread $PYTEST_ARGS > gpurun_out/pytest_gpu.log 2>&1 || { echo "gpu tests failed"; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
fi
timeout -k 10 600 python -u bench.py --steps 2 --recover-rounds ${C3_ROUNDS:-0} --c5-rounds 10000 --sync-rounds 0 --no-c1 --no-cpu-baseline --no-peak-detail --tables-out gpurun_out/c5_tables.json > gpurun_out/c5.json 2> gpurun_out/c5.err || { echo "bench failed"; tail -30 gpurun_out/c5.err; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/c5.json').read().strip().splitlines()[-1]); a=d['adversarial']; r=d.get('recover') or {}
print('head', d['value'], 'C3', r.get('value'), 'C5', a['value'], a['s_per_step'], a['roofline']['frac'], a['roofline']['kernel_avg_us'])"
