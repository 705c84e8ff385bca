#!/bin/bash
# Round-5 A/B of library builds on the headline and the keyed lines (C3, verify-all, C5): CONFIGS name:lib=<file> or
# name: (the in-tree library), each through one bench.py run.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for cfg in ${CONFIGS:-base:}; do
  name=${cfg%%:*}; kv=${cfg#*:}; envs=""
  case "$kv" in
    lib=*) envs="DRAND_GPU_LIB=${kv#lib=}";;
  esac
  env $envs timeout -k 10 400 python -u bench.py --steps ${BENCH_STEPS:-20} --sync-rounds 0 --no-c1 --no-cpu-baseline \
    --no-peak-detail --no-vp-negative --neg-steps 0 > gpurun_out/ab_$name.json 2> gpurun_out/ab_$name.err \
    || { echo "bench $name failed"; tail -20 gpurun_out/ab_$name.err; exit 1; }
  python3 -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], 'head', d['value'], 'c3', (d.get('recover') or {}).get('value'), 'va', (d.get('c2_verify_all') or {}).get('value'), 'c5', (d.get('adversarial') or {}).get('value'))" gpurun_out/ab_$name.json $name
done
