#!/bin/bash
# C5 A/B of environment switches, each argument "NAME|ENV=V,...": the adversarial Recover line alone (headline 1
# step); prints recovers/s and the per-item kernel's average launch.  Stops at the first failure.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
F="--steps 1 --warmup 1 --recover-rounds 0 --c5-rounds 10000 --sync-rounds 0 --no-c1 --no-cpu-baseline --no-peak-detail"
for a in "$@"; do
  IFS='|' read -r v envs <<< "$a"
  env ${envs//,/ } timeout -k 10 300 python bench.py $F --tables-out gpurun_out/abc5_${v}_tables.json > gpurun_out/abc5_$v.json 2> gpurun_out/abc5_$v.err || { tail -20 gpurun_out/abc5_$v.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/abc5_$v.json').read().strip().splitlines()[-1]); a=d['adversarial']
print('%-8s C5 %.0f recovers/s  %.3f s  per-item launch %.0f us  frac %.3f' % ('$v', a['value'], a['s_per_step'], a['roofline']['kernel_avg_us'], a['roofline']['frac']), flush=True)"
done
