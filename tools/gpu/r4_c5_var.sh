#!/bin/bash
# C5 line alone with variant libraries (tools/variants/libdrandgpu_<name>.so, names in VARS) and the built library;
# prints each run's C5 value and the pipeline's per-kernel time shares.  Stops at the first failure.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
C5="--steps 2 --warmup 1 --recover-rounds 0 --sync-rounds 0 --no-c1 --no-cpu-baseline --no-peak-detail"
for v in base $VARS; do
  if [ $v = base ]; then unset DRAND_GPU_LIB; else export DRAND_GPU_LIB=$PWD/tools/variants/libdrandgpu_$v.so; fi
  timeout -k 10 400 python -u bench.py $C5 --tables-out gpurun_out/c5v_${v}_tables.json > gpurun_out/c5v_$v.json 2> gpurun_out/c5v_$v.err || { echo "c5 $v failed"; tail -30 gpurun_out/c5v_$v.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/c5v_$v.json').read().strip().splitlines()[-1]); a=d['adversarial']
t=json.load(open('gpurun_out/c5v_${v}_tables.json'))['adversarial']
r=t['roofline']; print('$v', a['value'], a['s_per_step'], r.get('kernel'), round(r.get('frac') or 0, 4), r.get('kernel_avg_us'))
print(json.dumps(r.get('per_kernel_share')))
print(json.dumps({k: v for k, v in t['kernel_avg_us'].items() if k.startswith('k_ck') or k in ('k_verify_groups', 'k_rs_sac')}))"
done
