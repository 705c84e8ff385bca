#!/bin/bash
# C5 A/B: group tests (default) against one check per share (DG_GROUP=1), after the Recover/group GPU tests.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
PYTEST_K="recover or large_group or adversarial or group or golden" C5=1 BENCH_STEPS=5 bash tools/gpu/quick.sh || exit 1
DG_GROUP=1 timeout -k 10 300 python bench.py --steps 1 --warmup 1 --recover-rounds 0 --c5-rounds 10000 --sync-rounds 0 --no-c1 --no-cpu-baseline > gpurun_out/bench_c5_g1.json 2> gpurun_out/bench_c5_g1.err || exit 1
python3 - <<'PY'
import json
for f in ("gpurun_out/bench_c5.json", "gpurun_out/bench_c5_g1.json"):
    a = json.loads(open(f).read().strip().splitlines()[-1])["adversarial"]
    r = a.get("roofline") or {}
    print(f, "%.0f/s" % a["value"], "s/step %.3f" % a["s_per_step"], "verify frac %.3f" % r.get("frac", 0), r.get("checks_by_members"))
PY
