#!/bin/bash
# Round-2 profiles: rocprofv3 --kernel-trace --stats of the headline (overlapped and --sync), of Recover at C3
# (100k rounds, n=64) and of the adversarial Recover at C5 (10k rounds, n=256, 10% corrupted); then PMC passes,
# each counter group its own run: HBM-side bytes (FETCH_SIZE, WRITE_SIZE) of the --sync headline, C3 and C5,
# and the instruction mix / wave cycles of the C5 run.  Stops at the first failure.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r2prof
mkdir -p $O
export TMPDIR=/tmp
NOHEAD="--no-cpu-baseline --no-c1 --sync-rounds 0"
HEAD="$NOHEAD --recover-rounds 0 --c5-rounds 0"
C3="$NOHEAD --steps 1 --warmup 1 --recover-rounds 100000 --c5-rounds 0"
C5="$NOHEAD --steps 1 --warmup 1 --recover-rounds 0 --c5-rounds 10000"
cd /tmp
run() {  # name limit args...
  local name=$1 lim=$2
  shift 2
  echo "[profile] $name" >&2
  timeout -k 10 $lim rocprofv3 "$@" > $O/$name.log 2>&1 || { echo "$name failed"; tail -20 $O/$name.log; exit 1; }
}
run stats_async 300 --kernel-trace --stats --output-format csv -d $O/stats_async -o run -- python3 $R/bench.py $HEAD --steps 20
run stats_sync 300 --kernel-trace --stats --output-format csv -d $O/stats_sync -o run -- python3 $R/bench.py $HEAD --sync --steps 10
run stats_c3 300 --kernel-trace --stats --output-format csv -d $O/stats_c3 -o run -- python3 $R/bench.py $C3
run stats_c5 300 --kernel-trace --stats --output-format csv -d $O/stats_c5 -o run -- python3 $R/bench.py $C5
for c in FETCH_SIZE WRITE_SIZE; do
  echo "[profile] pmc $c" >&2
  timeout -s KILL 200 rocprofv3 --pmc $c --output-format csv -d $O/pmc_head_$c -o run -- python3 $R/bench.py $HEAD --sync --steps 1 --warmup 1 > $O/pmc_head_$c.log 2>&1 || { echo "pmc head $c failed"; tail -5 $O/pmc_head_$c.log; exit 1; }
  timeout -s KILL 200 rocprofv3 --pmc $c --output-format csv -d $O/pmc_c3_$c -o run -- python3 $R/bench.py $C3 > $O/pmc_c3_$c.log 2>&1 || { echo "pmc c3 $c failed"; tail -5 $O/pmc_c3_$c.log; exit 1; }
  timeout -s KILL 200 rocprofv3 --pmc $c --output-format csv -d $O/pmc_c5_$c -o run -- python3 $R/bench.py $C5 > $O/pmc_c5_$c.log 2>&1 || { echo "pmc c5 $c failed"; tail -5 $O/pmc_c5_$c.log; exit 1; }
done
for c in "SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES" "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU"; do
  tag=$(echo $c | cut -d' ' -f1)
  echo "[profile] pmc $tag" >&2
  timeout -s KILL 200 rocprofv3 --pmc $c --output-format csv -d $O/pmc_c5_$tag -o run -- python3 $R/bench.py $C5 > $O/pmc_c5_$tag.log 2>&1 || { echo "pmc c5 $tag failed"; tail -5 $O/pmc_c5_$tag.log; exit 1; }
done
find $O -name "*.csv" | sort
