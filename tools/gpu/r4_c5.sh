#!/bin/bash
# Round-4 C5 A/B: every -m gpu test (SKIP_TESTS=1 skips), then the C5 line alone with the pairing-check pipeline
# (checks.h) and with the round-3 single-lane kernel (DG_CK_OLD=1); stops at the first failure.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
if [ -z "$SKIP_TESTS" ]; then
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/pytest_gpu.log 2>&1 || { echo "gpu tests failed"; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
fi
C5="--steps 2 --warmup 1 --recover-rounds 0 --sync-rounds 0 --no-c1 --no-cpu-baseline --no-peak-detail"
for v in ${VARIANTS:-new old}; do
  if [ $v = old ]; then export DG_CK_OLD=1; else unset DG_CK_OLD; fi
  timeout -k 10 400 python -u bench.py $C5 --tables-out gpurun_out/c5_${v}_tables.json > gpurun_out/c5_$v.json 2> gpurun_out/c5_$v.err || { echo "c5 $v failed"; tail -30 gpurun_out/c5_$v.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/c5_$v.json').read().strip().splitlines()[-1]); a=d['adversarial']; print('$v', a['value'], a['s_per_step'], json.dumps(a['roofline']))"
  python3 -c "import json; d=json.load(open('gpurun_out/c5_${v}_tables.json')); print(json.dumps(d['adversarial']['kernel_avg_us']))"
done
