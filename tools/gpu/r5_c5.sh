#!/bin/bash
# Round-5: C5 (adversarial Recover) line and its kernel stats, after a pipeline change (GPU tests of Recover first).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread -k "recover or partial or c5 or corrupt" \
    > gpurun_out/c5_pytest.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/c5_pytest.log; exit 1; }
  tail -2 gpurun_out/c5_pytest.log
fi
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c5p -o run -- \
  python3 -u bench.py --steps 2 --recover-rounds 0 --sync-rounds 0 --no-c1 --no-cpu-baseline --no-peak-detail \
  --no-vp-negative --neg-steps 0 > gpurun_out/c5p.json 2> gpurun_out/c5p.err || { echo "c5 failed"; tail -20 gpurun_out/c5p.err; exit 1; }
grep -E '"k_ck_miller"|"k_ck_expsq"|"k_ck_expdec"|"k_rs_sac"|"k_ck_lines2"|"k_ck_sub"|"k_rs_digits"' gpurun_out/c5p/run_kernel_stats.csv
python3 -c "import json; d=json.loads(open('gpurun_out/c5p.json').read().strip().splitlines()[-1]); a=d.get('adversarial') or {}; print('c5', a.get('value'), a.get('unit'))"
