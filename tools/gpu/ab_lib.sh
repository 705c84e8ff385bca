#!/bin/bash
# A/B of a variant library (tools/variants/libdrandgpu_$1.so) against the built one on the Recover lines
# (C3 100k rounds, C5 10k rounds); stops at the first failure.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
F="--steps 1 --warmup 1 --recover-rounds 100000 --c5-rounds 10000 --sync-rounds 0 --no-c1 --no-cpu-baseline"
timeout -k 10 400 python bench.py $F > gpurun_out/ab_base.json 2> gpurun_out/ab_base.err || { tail -20 gpurun_out/ab_base.err; exit 1; }
DRAND_GPU_LIB=$PWD/tools/variants/libdrandgpu_$1.so timeout -k 10 400 python bench.py $F > gpurun_out/ab_var.json 2> gpurun_out/ab_var.err || { tail -20 gpurun_out/ab_var.err; exit 1; }
python3 - <<'PY'
import json
for f in ("gpurun_out/ab_base.json", "gpurun_out/ab_var.json"):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    r, a = d["recover"], d["adversarial"]
    print(f, "C3 %.0f/s terms %.0f us" % (r["value"], r["kernel_avg_us"].get("k_recover_terms", 0)),
          "C5 %.0f/s terms %.0f us verify %.0f us" % (a["value"], a["kernel_avg_us"].get("k_recover_terms", 0),
                                                    a["kernel_avg_us"].get("k_verify_groups", 0)))
PY
