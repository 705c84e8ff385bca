#!/bin/bash
# Per-dispatch cost of kernels with a private segment under the HSA runtime's scratch settings (tooling):
# tools/microbench/launch_cost under each environment variant -> gpurun_out/scratch_env.txt
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
o=gpurun_out/scratch_env.txt
: > $o
for v in "default:" "noreclaim:HSA_NO_SCRATCH_RECLAIM=1" "noasync:HSA_ENABLE_SCRATCH_ASYNC_RECLAIM=0" "both:HSA_NO_SCRATCH_RECLAIM=1,HSA_ENABLE_SCRATCH_ASYNC_RECLAIM=0"; do
  name=${v%%:*}; envs=${v#*:}
  echo "== $name" >> $o
  env $(echo $envs | tr ',' ' ') timeout -k 10 120 tools/microbench/launch_cost >> $o 2>&1 || exit 1
done
cat $o
