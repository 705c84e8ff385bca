#!/bin/bash
# Round-5: keyed-batch (Recover / VerifyPartial) change -- their GPU tests, then the C3 / C5 / verify-all lines
# (no headline profile) and a kernel-stats trace of the same run.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread -k "recover or partial or c5 or corrupt" \
    > gpurun_out/keyed_pytest.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/keyed_pytest.log; exit 1; }
  tail -2 gpurun_out/keyed_pytest.log
fi
timeout -k 10 600 python3 -u bench.py --steps 3 --sync-rounds 0 --no-c1 --no-cpu-baseline --no-peak-detail \
  --no-vp-negative --neg-steps 0 > gpurun_out/keyed.json 2> gpurun_out/keyed.err || { echo "bench failed"; tail -20 gpurun_out/keyed.err; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/keyed.json').read().strip().splitlines()[-1])
print('head', d['value'])
for k in ('recover','c2_verify_all','adversarial'): print(k, (d.get(k) or {}).get('value'))"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/keyedp -o run -- \
  python3 -u bench.py --steps 2 --sync-rounds 0 --no-c1 --no-cpu-baseline --no-peak-detail \
  --no-vp-negative --neg-steps 0 > gpurun_out/keyedp.json 2> gpurun_out/keyedp.err || { echo "profile failed"; tail -20 gpurun_out/keyedp.err; exit 1; }
grep -E '"k_key_combine"|"k_key_accum"|"k_rs_combine"|"k_rs_digits"|"k_rs_sac"' gpurun_out/keyedp/run_kernel_stats.csv
