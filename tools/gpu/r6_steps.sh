#!/bin/bash
# Round-6: the headline's per-step completion times (BENCH_STEP_TIMES=1): fill, steady spacing and drain of the driver's
# 20-step region, then a 40-step region.  VARIANTS: "name:ENV=VAL,ENV=VAL ..." (default "base:")
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
HEAD="--gpus 1 --warmup 5 --recover-rounds 0 --c5-rounds 0 --sync-rounds 0 --no-c1 --no-cpu-baseline --neg-steps ${NEG_STEPS:-0} --no-peak-detail --no-kernel-timing"
for v in ${VARIANTS:-base:}; do
  name=${v%%:*}; envs=${v#*:}; envs=${envs//,/ }
  for st in ${STEPS:-20 40}; do
    env $envs BENCH_STEP_TIMES=1 timeout -k 10 300 python -u bench.py $HEAD --steps $st --tables-out gpurun_out/st_${name}_$st.tables.json \
      > gpurun_out/st_${name}_$st.json 2> gpurun_out/st_${name}_$st.err || { echo "bench $name $st failed"; tail -20 gpurun_out/st_${name}_$st.err; exit 1; }
    python3 - gpurun_out/st_${name}_$st.json gpurun_out/st_${name}_$st.err $name $st <<'PY'
import json, sys, re
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
line = [l for l in open(sys.argv[2]) if l.startswith("[step_times]")][-1]
ts = json.loads(line.split("completions (ms): ")[1])
gaps = [round(b - a, 2) for a, b in zip(ts, ts[1:])]
neg = d.get("c2_negative") or {}
print(sys.argv[3], sys.argv[4], "value %.4g ms/step %.3f" % (d["value"], d["ms_per_step"]), "first %.2f last %.2f" % (ts[0], ts[-1]),
      "gaps", gaps, "neg", neg.get("value"))
PY
  done
done
