#!/bin/bash
# C3 A/B of variant libraries (tools/variants/libdrandgpu_<name>.so) against the built one, alternating twice: the
# Recover line alone (headline 1 step); prints recovers/s and the top kernels.  Stops at the first failure.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
F="--steps 1 --warmup 1 --recover-rounds 100000 --c5-rounds 0 --sync-rounds 0 --no-c1 --no-cpu-baseline --no-peak-detail"
for rep in 1 2; do
for v in base "$@"; do
  L=""
  [ "$v" != base ] && L=$PWD/tools/variants/libdrandgpu_$v.so
  env ${L:+DRAND_GPU_LIB=$L} timeout -k 10 300 python bench.py $F --tables-out gpurun_out/abc3_${v}_tables.json > gpurun_out/abc3_$v.json 2> gpurun_out/abc3_$v.err || { tail -20 gpurun_out/abc3_$v.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/abc3_$v.json').read().strip().splitlines()[-1]); a=d['recover']
t=json.load(open('gpurun_out/abc3_${v}_tables.json'))['recover']['kernel_avg_us']
top={k: round(x) for k, x in sorted(t.items(), key=lambda kv: -kv[1])[:6]}
print('%-8s C3 %.0f recovers/s  %.4f s  %s' % ('$v', a['value'], a['s_per_step'], top), flush=True)"
done
done
