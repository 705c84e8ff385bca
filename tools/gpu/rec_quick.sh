#!/bin/bash
# Recover lines only (C3 100k rounds, C5 10k rounds) after the Recover GPU tests; stops at the first failure.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "${PYTEST_K:-recover or group or large_group or adversarial}" > gpurun_out/pytest_rec.log 2>&1 || { echo "gpu tests failed"; tail -30 gpurun_out/pytest_rec.log; exit 1; }
tail -1 gpurun_out/pytest_rec.log
timeout -k 10 400 python bench.py --steps 1 --warmup 1 --recover-rounds 100000 --c5-rounds 10000 --sync-rounds 0 --no-c1 --no-cpu-baseline > gpurun_out/rec.json 2> gpurun_out/rec.err || { tail -20 gpurun_out/rec.err; exit 1; }
python3 - <<'PY'
import json
d = json.loads(open("gpurun_out/rec.json").read().strip().splitlines()[-1])
r, a = d["recover"], d["adversarial"]
print("C3 %.0f/s (host API %.0f/s) terms %.0f us kmsm %.0f us" % (r["value"], r["host_api_value"], r["kernel_avg_us"].get("k_recover_terms", 0), r["kernel_avg_us"].get("k_kmsm_chunks", 0)))
print("C5 %.0f/s terms %.0f us verify %.0f us" % (a["value"], a["kernel_avg_us"].get("k_recover_terms", 0), a["kernel_avg_us"].get("k_verify_groups", 0)))
print(sorted(r["kernel_avg_us"].items(), key=lambda x: -x[1])[:8])
PY
