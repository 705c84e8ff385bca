#!/bin/bash
# Round-5 verdict item 6: one rank's load at N = 8 (--global-rounds 125000: one batch of 125k rounds per step) on one
# GPU against the N = 1 headline (100k rounds per step), per-round rate within 5%.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
F="--steps 30 --recover-rounds 0 --c5-rounds 0 --sync-rounds 0 --no-c1 --no-cpu-baseline --no-peak-detail --no-vp-negative --neg-steps 0"
timeout -k 10 300 python -u bench.py $F > gpurun_out/scale1_n1.json 2> gpurun_out/scale1_n1.err || { echo "n1 failed"; tail -20 gpurun_out/scale1_n1.err; exit 1; }
timeout -k 10 300 python -u bench.py $F --global-rounds 125000 > gpurun_out/scale1_125k.json 2> gpurun_out/scale1_125k.err || { echo "125k failed"; tail -20 gpurun_out/scale1_125k.err; exit 1; }
python3 - <<'PY'
import json
a = json.loads(open("gpurun_out/scale1_n1.json").read().strip().splitlines()[-1])
b = json.loads(open("gpurun_out/scale1_125k.json").read().strip().splitlines()[-1])
print("n1", a["value"], a["config"]["batches_per_gpu"], "125k", b["value"], b["config"]["batches_per_gpu"], "ratio", round(b["value"] / a["value"], 4))
PY
