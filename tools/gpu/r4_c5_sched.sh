#!/bin/bash
# C5 line alone under several pass schedules of Recover's pairing-check pipeline (DG_CK_PASSES / DG_CK_MARGIN0 /
# DG_CK_MARGIN), each run printing its checks per pass (DG_CK_TRACE) and the C5 value.  Stops at the first failure.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
C5="--steps 2 --warmup 1 --recover-rounds 0 --sync-rounds 0 --no-c1 --no-cpu-baseline --no-peak-detail --no-kernel-timing"
for s in ${SCHEDS:-8:6:2}; do
  IFS=: read P M0 M <<< "$s"
  DG_CK_TRACE=1 DG_CK_PASSES=$P DG_CK_MARGIN0=$M0 DG_CK_MARGIN=$M timeout -k 10 400 python -u bench.py $C5 --tables-out gpurun_out/c5s_tables.json > gpurun_out/c5s_$s.json 2> gpurun_out/c5s_$s.err || { echo "c5 $s failed"; tail -30 gpurun_out/c5s_$s.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/c5s_$s.json').read().strip().splitlines()[-1]); a=d['adversarial']
print('sched $s', a['value'], a['s_per_step'])"
  grep "prefix pass" gpurun_out/c5s_$s.err | tail -${P:-8} | tr '\n' ' '; echo
done
