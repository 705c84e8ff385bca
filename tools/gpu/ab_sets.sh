#!/bin/bash
# A/B of the overlapped pipeline depth: workspace sets (DG_SETS) with as many status buffers in flight.
# (GPU_MAX_HW_QUEUES stays at the box's 4: 8 hardware queues per process fail with
# HSA_STATUS_ERROR_OUT_OF_RESOURCES there.)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
F="--steps 20 --recover-rounds 0 --c5-rounds 0 --sync-rounds 0 --no-c1 --no-cpu-baseline --no-kernel-timing"
for s in 4 6 8 3; do
  DG_SETS=$s timeout -k 10 200 python -u bench.py $F --status-bufs $s > gpurun_out/abs_$s.json 2>gpurun_out/abs_$s.err || { tail -5 gpurun_out/abs_$s.err; exit 1; }
  python3 -c "import json;d=json.loads(open('gpurun_out/abs_$s.json').read().strip().splitlines()[-1]);print('sets $s', '%.0f'%d['value'], '%.2f ms'%d['ms_per_step'])"
done
