#!/bin/bash
# Round-5: host launch cost under load -- headline + c2_negative with HIP_FORCE_DEV_KERNARG unset / 0 (kernel arguments
# in device memory written over PCIe vs in host memory), host enqueue time reported by bench.py.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
for kv in ${KVS:-default 0}; do
  if [ "$kv" = default ]; then envs=""; else envs="HIP_FORCE_DEV_KERNARG=$kv"; fi
  env $envs DG_XR_SKIP=${DG_XR_SKIP:-1} DG_BENCH_HOSTPROF=1 timeout -k 10 300 python -u bench.py --steps 20 \
    --recover-rounds 0 --c5-rounds 0 --sync-rounds 0 --no-c1 --no-cpu-baseline --no-peak-detail --no-vp-negative \
    --neg-steps 10 > gpurun_out/karg_$kv.json 2> gpurun_out/karg_$kv.err \
    || { echo "bench $kv failed"; tail -20 gpurun_out/karg_$kv.err; exit 1; }
  grep hostprof gpurun_out/karg_$kv.err
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); n=d['c2_negative']; print('kernarg', sys.argv[2], 'head', d['value'], d['ms_per_step'], 'neg', n['value'], n['ms_per_step'])" gpurun_out/karg_$kv.json $kv
done
