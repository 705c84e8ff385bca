#!/bin/bash
# Round-5: C5 line A/B over environment configurations (CONFIGS="name:VAR=v,VAR2=w ...").
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for cfg in $CONFIGS; do
  name=${cfg%%:*}; kv=${cfg#*:}; envs="${kv//,/ }"
  env $envs timeout -k 10 400 python -u bench.py --steps 2 --recover-rounds 0 --sync-rounds 0 --no-c1 --no-cpu-baseline \
    --no-peak-detail --no-vp-negative --neg-steps 0 --no-kernel-timing > gpurun_out/c5ab_$name.json 2> gpurun_out/c5ab_$name.err \
    || { echo "c5 $name failed"; tail -20 gpurun_out/c5ab_$name.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); a=d.get('adversarial') or {}; print(sys.argv[2], 'c5', a.get('value'), a.get('unit'))" gpurun_out/c5ab_$name.json $name
done
