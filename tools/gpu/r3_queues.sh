#!/bin/bash
# The configuration that aborted in round 2 (6 workspace sets, 8 hardware queues per process), once: the headline
# and the C5 adversarial Recover (whose per-item pass dispatches the largest private segment), logs kept.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
GPU_MAX_HW_QUEUES=8 DG_SETS=6 timeout -k 10 400 python -u bench.py --steps 8 --no-cpu-baseline --no-c1 --sync-rounds 0 --recover-rounds 0 --c5-rounds 10000 --tables-out gpurun_out/q8s6_tables.json > gpurun_out/q8s6.json 2> gpurun_out/q8s6.err || { echo "q8s6 failed"; tail -30 gpurun_out/q8s6.err; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/q8s6.json').read().strip().splitlines()[-1]); print('q8s6 ok', d['value'], (d.get('adversarial') or {}).get('value'))"
