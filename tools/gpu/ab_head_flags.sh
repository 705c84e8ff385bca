#!/bin/bash
# Headline A/B of bench / environment settings, each argument "NAME|ENV=V,...|--bench --flags" (either part may be
# empty); 30 overlapped steps each; stops at the first failure.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
F="--steps ${AB_STEPS:-30} --warmup 1 --recover-rounds 0 --c5-rounds 0 --sync-rounds 0 --no-c1 --no-cpu-baseline --no-peak-detail --no-kernel-timing"
for a in "$@"; do
  IFS='|' read -r n envs flags <<< "$a"
  env ${envs//,/ } timeout -k 10 300 python bench.py $F $flags --tables-out gpurun_out/abf_${n}_tables.json > gpurun_out/abf_$n.json 2> gpurun_out/abf_$n.err || { tail -20 gpurun_out/abf_$n.err; exit 1; }
  python3 -c "
import json; d = json.loads(open('gpurun_out/abf_$n.json').read().strip().splitlines()[-1])
print('%-12s %.0f rounds/s  %.3f ms/step' % ('$n', d['value'], d['ms_per_step']), flush=True)"
done
