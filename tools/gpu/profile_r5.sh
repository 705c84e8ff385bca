#!/bin/bash
# Round-5 profiles: rocprofv3 --kernel-trace --stats of the headline (overlapped and --sync), of Recover at C3
# (100k rounds, n=64) and of the adversarial Recover at C5 (10k rounds, n=256, 10% corrupted); then PMC passes,
# each counter group its own run and config (CONFIGS, default "head c3 c5"): HBM-side bytes (FETCH_SIZE, WRITE_SIZE), VALU instruction counts and
# wave cycles (SQ_*), GRBM_GUI_ACTIVE (the clock).  Stops at the first failure.  PASSES=stats|pmc|all (default all)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5prof
mkdir -p $O
export TMPDIR=/tmp
NOHEAD="--no-cpu-baseline --no-c1 --sync-rounds 0 --no-peak-detail --no-vp-negative --tables-out $O/tables.json"
HEAD="$NOHEAD --recover-rounds 0 --c5-rounds 0 --neg-steps 0"
C3="$NOHEAD --neg-steps 0 --steps 1 --warmup 1 --recover-rounds 100000 --c5-rounds 0"
C5="$NOHEAD --neg-steps 0 --steps 1 --warmup 1 --recover-rounds 0 --c5-rounds 10000"
NEG="$HEAD --steps 2 --warmup 1 --neg-steps 3 --no-vp-negative --no-kernel-timing"
P=${PASSES:-all}
cd /tmp
run() {  # name limit args...
  local name=$1 lim=$2
  shift 2
  echo "[profile] $name" >&2
  timeout -k 10 $lim rocprofv3 "$@" > $O/$name.log 2>&1 || { echo "$name failed"; tail -20 $O/$name.log; exit 1; }
}
if [ "$P" = all ] || [ "$P" = stats ]; then
for cfg in ${CONFIGS:-head c3 c5}; do case $cfg in
head)
run stats_async 300 --kernel-trace --stats --output-format csv -d $O/stats_async -o run -- python3 $R/bench.py $HEAD --steps 20
run stats_sync 300 --kernel-trace --stats --output-format csv -d $O/stats_sync -o run -- python3 $R/bench.py $HEAD --sync --steps 10;;
c3)
run stats_c3 300 --kernel-trace --stats --output-format csv -d $O/stats_c3 -o run -- python3 $R/bench.py $C3;;
c5)
run stats_c5 300 --kernel-trace --stats --output-format csv -d $O/stats_c5 -o run -- python3 $R/bench.py $C5;;
neg)
run stats_neg 300 --kernel-trace --stats --output-format csv -d $O/stats_neg -o run -- python3 $R/bench.py $NEG;;
esac; done
fi
if [ "$P" = all ] || [ "$P" = pmc ]; then
pmc() {  # tag counters config-name config-args
  local tag=$1 ctr=$2 cfg=$3
  shift 3
  echo "[profile] pmc $cfg $tag" >&2
  timeout -s KILL 240 rocprofv3 --pmc $ctr --output-format csv -d $O/pmc_${cfg}_$tag -o run -- python3 $R/bench.py "$@" > $O/pmc_${cfg}_$tag.log 2>&1 || { echo "pmc $cfg $tag failed"; tail -5 $O/pmc_${cfg}_$tag.log; exit 1; }
}
for cfg in ${CONFIGS:-head c3 c5}; do
  case $cfg in head) A="$HEAD --sync --steps 1 --warmup 1";; c3) A="$C3";; c5) A="$C5";;
    c2neg) A="$HEAD --steps 1 --warmup 1 --neg-steps 2";; esac
  pmc FETCH_SIZE FETCH_SIZE $cfg $A
  pmc WRITE_SIZE WRITE_SIZE $cfg $A
  pmc SQ_VALU "SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAVES" $cfg $A
  pmc SQ_MEM "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_INSTS_SALU" $cfg $A
  pmc GRBM "GRBM_GUI_ACTIVE GRBM_COUNT" $cfg $A
done
# the per-dispatch CSVs exceed what a call can bring back: summarise on the box, keep the summaries only
cp $R/profiles/traffic.json $O/traffic.json 2>/dev/null
python3 $R/tools/traffic.py $O $O/pmc_summary.csv $O/traffic.json > $O/traffic.log 2>&1 || { echo "summary failed"; tail -5 $O/traffic.log; exit 1; }
rm -rf $O/pmc_*/
fi
find $O -name "*.csv" | sort
