#!/bin/bash
# Headline A/B of variant libraries (tools/variants/libdrandgpu_<name>.so, built by tools/build_variant.sh)
# against the built one: AB_STEPS (30) overlapped steps each, the isolated times of the top kernels from the side
# tables; stops at the first failure.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
F="--steps ${AB_STEPS:-30} --warmup 1 --recover-rounds 0 --c5-rounds 0 --sync-rounds 0 --no-c1 --no-cpu-baseline --no-peak-detail"
for v in base "$@"; do
  L=""
  [ "$v" != base ] && L=$PWD/tools/variants/libdrandgpu_$v.so
  env ${L:+DRAND_GPU_LIB=$L} timeout -k 10 300 python bench.py $F --tables-out gpurun_out/ab_${v}_tables.json > gpurun_out/ab_$v.json 2> gpurun_out/ab_$v.err || { tail -20 gpurun_out/ab_$v.err; exit 1; }
  python3 - $v <<'PY'
import json, sys
v = sys.argv[1]
d = json.loads(open("gpurun_out/ab_%s.json" % v).read().strip().splitlines()[-1])
t = json.load(open("gpurun_out/ab_%s_tables.json" % v))
iso, ov = t["kernel_avg_us_isolated"], t["kernel_avg_us"]
top = {k: (round(iso[k]), round(ov.get(k, 0))) for k in sorted(iso, key=lambda k: -iso[k])[:6]}
print("%-8s %.0f rounds/s  %.3f ms/step  iso/ovl %s" % (v, d["value"], d["ms_per_step"], top), flush=True)
PY
done
