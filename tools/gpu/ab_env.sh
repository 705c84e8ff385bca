#!/bin/bash
# A/B of library environment switches on the headline (blocking batches: per-kernel isolated times).  Each argument
# is NAME or NAME:VAR=VALUE[,VAR=VALUE]; stops at the first failure.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
F="--steps ${AB_STEPS:-8} --warmup 1 --recover-rounds 0 --c5-rounds 0 --sync-rounds 0 --no-c1 --no-cpu-baseline $AB_FLAGS"
names=()
for a in "$@"; do
  n=${a%%:*}
  envs=""
  [[ "$a" == *:* ]] && envs=${a#*:}
  names+=("$n")
  env ${envs//,/ } timeout -k 10 300 python bench.py $F > gpurun_out/ab_$n.json 2> gpurun_out/ab_$n.err || { tail -20 gpurun_out/ab_$n.err; exit 1; }
done
python3 - "${names[@]}" <<'PY'
import json, sys
for v in sys.argv[1:]:
    d = json.loads(open("gpurun_out/ab_%s.json" % v).read().strip().splitlines()[-1])
    iso, ov = d["kernel_avg_us_isolated"], d["kernel_avg_us"]
    msm = {k: round(t) for k, t in iso.items() if "msm" in k or "sum_rows" in k or "binv" in k}
    print("%-10s %.0f rounds/s  %.2f ms/step  fallbacks %s" % (v, d["value"], d["ms_per_step"], d.get("batch_fallbacks")))
    print("    iso", msm)
PY
