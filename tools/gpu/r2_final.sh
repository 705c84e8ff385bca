#!/bin/bash
# Round-end evidence: every GPU test, smoke(), the full default bench, then the round-2 profiles
# (tools/gpu/profile_r2.sh); stops at the first failure.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
BENCH_STEPS=30 bash tools/gpu/r2_check.sh || exit 1
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
bash tools/gpu/profile_r2.sh
