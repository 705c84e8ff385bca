#!/bin/bash
# A/B of variant libraries (tools/variants/libdrandgpu_<name>.so, args) against the built one on the headline
# (blocking batches: per-kernel isolated times); stops at the first failure.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
F="--steps 6 --warmup 1 --recover-rounds 0 --c5-rounds 0 --sync-rounds 0 --no-c1 --no-cpu-baseline"
timeout -k 10 300 python bench.py $F > gpurun_out/ab_base.json 2> gpurun_out/ab_base.err || { tail -20 gpurun_out/ab_base.err; exit 1; }
for v in "$@"; do
  DRAND_GPU_LIB=$PWD/tools/variants/libdrandgpu_$v.so timeout -k 10 300 python bench.py $F > gpurun_out/ab_$v.json 2> gpurun_out/ab_$v.err || { tail -20 gpurun_out/ab_$v.err; exit 1; }
done
python3 - "$@" <<'PY'
import json, sys
for v in ["base"] + sys.argv[1:]:
    d = json.loads(open("gpurun_out/ab_%s.json" % v).read().strip().splitlines()[-1])
    iso, ov = d["kernel_avg_us_isolated"], d["kernel_avg_us"]
    print("%-12s %.0f rounds/s  chunks iso %.0f us ovl %.0f us  buckets %.0f" % (v, d["value"], iso.get("k_msm_chunks", 0),
          ov.get("k_msm_chunks", 0), iso.get("k_msm_buckets", 0)))
PY
