#!/bin/bash
# C5 sub-lines, the built library against an alternate one (A/B on one box): LINES="c5 c5vp", ALT=<path to .so>
set -o pipefail
mkdir -p gpurun_out
ALT=${ALT:-drand_amd/ab/libdrandgpu_m0.so}
for line in ${LINES:-c5 c5vp}; do
  timeout -k 10 300 python3 -u tools/prof_lines.py $line --calls ${CALLS:-3} > gpurun_out/ab_${line}_new.log 2>&1 || exit 1
  DRAND_GPU_LIB=$ALT timeout -k 10 300 python3 -u tools/prof_lines.py $line --calls ${CALLS:-3} > gpurun_out/ab_${line}_alt.log 2>&1 || exit 1
  echo "new: $(tail -1 gpurun_out/ab_${line}_new.log)"
  echo "alt: $(tail -1 gpurun_out/ab_${line}_alt.log)"
done
