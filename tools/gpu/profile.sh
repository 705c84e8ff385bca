#!/bin/bash
# Full bench (CPU baseline + Recover), rocprofv3 kernel stats of the bench command, PMC passes (HBM traffic,
# instruction mix) -- each pass its own run; stops at the first failure.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 500 python -u bench.py > gpurun_out/bench_full.json 2> gpurun_out/bench_full.err || { echo "bench failed"; tail -20 gpurun_out/bench_full.err; exit 1; }
tail -1 gpurun_out/bench_full.json | cut -c1-300
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof/stats -o run -- python3 $R/bench.py --no-cpu-baseline --recover-rounds 0 --c5-rounds 0 --sync-rounds 0 > $R/gpurun_out/prof/stats.log 2>&1 || { echo "rocprof stats failed"; tail -20 $R/gpurun_out/prof/stats.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof/stats_sync -o run -- python3 $R/bench.py --sync --no-cpu-baseline --recover-rounds 0 --c5-rounds 0 --sync-rounds 0 > $R/gpurun_out/prof/stats_sync.log 2>&1 || { echo "rocprof stats (sync) failed"; tail -20 $R/gpurun_out/prof/stats_sync.log; exit 1; }
for c in FETCH_SIZE WRITE_SIZE "SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES" "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_WAIT_INST_ANY"; do
  tag=$(echo $c | cut -d' ' -f1)
  timeout -s KILL 240 rocprofv3 --pmc $c --output-format csv -d $R/gpurun_out/prof/pmc_$tag -o run -- python3 $R/bench.py --sync --steps 1 --warmup 1 --no-cpu-baseline --recover-rounds 0 --c5-rounds 0 --sync-rounds 0 > $R/gpurun_out/prof/pmc_$tag.log 2>&1 || { echo "pmc $c failed"; tail -5 $R/gpurun_out/prof/pmc_$tag.log; exit 1; }
done
find $R/gpurun_out/prof -name "*.csv" | head -20
