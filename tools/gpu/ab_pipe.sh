#!/bin/bash
# A/B of the overlapped pipeline: default, without the batch binding, with 3 status buffers.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
F="--steps 20 --recover-rounds 0 --c5-rounds 0 --sync-rounds 0 --no-c1 --no-cpu-baseline --no-kernel-timing"
for v in "A:" "B:DG_NO_BIND=1" "C:--status-bufs 3" "D:--sync"; do
  tag=${v%%:*}; arg=${v#*:}
  if [[ $arg == DG_* ]]; then env $arg timeout -k 10 200 python -u bench.py $F > gpurun_out/ab_$tag.json 2>gpurun_out/ab_$tag.err || exit 1
  else timeout -k 10 200 python -u bench.py $F $arg > gpurun_out/ab_$tag.json 2>gpurun_out/ab_$tag.err || exit 1; fi
  python3 -c "import json;d=json.loads(open('gpurun_out/ab_$tag.json').read().strip().splitlines()[-1]);print('$tag', '$arg', '%.0f'%d['value'], '%.2f ms'%d['ms_per_step'])"
done
