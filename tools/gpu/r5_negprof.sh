#!/bin/bash
# Round-5: isolation kernel latencies alone (one blocking failed batch at a time) and under the overlapped
# c2_negative steps (kernel traces), summarised by tools/trace/xr_lat.py.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/negp_single -o run -- \
  python3 -u tools/trace/neg_single.py 3 > gpurun_out/negp_single.log 2>&1 || { echo "single failed"; tail -20 gpurun_out/negp_single.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/negp_bench -o run -- \
  python3 -u bench.py --steps 2 --recover-rounds 0 --c5-rounds 0 --sync-rounds 0 --no-c1 --no-cpu-baseline \
  --no-peak-detail --no-vp-negative --neg-steps 5 --no-kernel-timing > gpurun_out/negp_bench.json 2> gpurun_out/negp_bench.err \
  || { echo "bench failed"; tail -20 gpurun_out/negp_bench.err; exit 1; }
python3 tools/trace/xr_lat.py gpurun_out/negp_single/run_kernel_trace.csv gpurun_out/negp_bench/run_kernel_trace.csv
if [ -n "$CUS" ]; then
  SKIP_TESTS=1 CONFIGS="base: $(for c in $CUS; do printf 'cus%s:DG_TAIL_CUS=%s ' $c $c; done)" bash tools/gpu/r5_lat.sh
fi
