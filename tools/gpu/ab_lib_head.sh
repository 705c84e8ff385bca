#!/bin/bash
# Headline A/B of variant libraries (tools/variants/libdrandgpu_<name>.so, built by tools/build_variant.sh)
# against the built one: 30 overlapped steps each, per-kernel isolated times; stops at the first failure.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
F="--steps ${AB_STEPS:-30} --warmup 1 --recover-rounds 0 --c5-rounds 0 --sync-rounds 0 --no-c1 --no-cpu-baseline"
timeout -k 10 300 python bench.py $F > gpurun_out/ab_base.json 2> gpurun_out/ab_base.err || { tail -20 gpurun_out/ab_base.err; exit 1; }
for v in "$@"; do
  DRAND_GPU_LIB=$PWD/tools/variants/libdrandgpu_$v.so timeout -k 10 300 python bench.py $F > gpurun_out/ab_$v.json 2> gpurun_out/ab_$v.err || { tail -20 gpurun_out/ab_$v.err; exit 1; }
done
python3 - base "$@" <<'PY'
import json, sys
for v in sys.argv[1:]:
    d = json.loads(open("gpurun_out/ab_%s.json" % v).read().strip().splitlines()[-1])
    iso, ov = d["kernel_avg_us_isolated"], d["kernel_avg_us"]
    top = {k: (round(iso[k]), round(ov.get(k, 0))) for k in sorted(iso, key=lambda k: -iso[k])[:8]}
    print("%-8s %.0f rounds/s  %.2f ms/step  iso/ovl %s" % (v, d["value"], d["ms_per_step"], top))
PY
