#!/bin/bash
# Headline A/B of environment switches (library or HIP runtime).  Each argument is NAME or NAME:VAR=VALUE[,VAR=VALUE];
# prints rounds/s per variant; stops at the first failure.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
F="--steps ${AB_STEPS:-20} --warmup 1 --recover-rounds 0 --c5-rounds 0 --sync-rounds 0 --no-c1 --no-cpu-baseline --no-peak-detail --no-kernel-timing $AB_FLAGS"
for a in "$@"; do
  n=${a%%:*}
  envs=""
  [[ "$a" == *:* ]] && envs=${a#*:}
  env ${envs//,/ } timeout -k 10 300 python bench.py $F --tables-out gpurun_out/ab_${n}_tables.json > gpurun_out/ab_$n.json 2> gpurun_out/ab_$n.err || { tail -20 gpurun_out/ab_$n.err; exit 1; }
  python3 -c "
import json, sys; d = json.loads(open('gpurun_out/ab_$n.json').read().strip().splitlines()[-1])
print('%-12s %.0f rounds/s  %.3f ms/step' % ('$n', d['value'], d['ms_per_step']), flush=True)"
done
