#!/bin/bash
# Round-6 profiles.  PASSES (default "trace stats pmc"):
#   trace  rocprofv3 --kernel-trace of the driver's headline (20 steps, 5 warmup): the per-dispatch CSV (timeline of
#          the timed region: fill, drain) -> gpurun_out/r6prof/head_trace.csv
#   stats  rocprofv3 --kernel-trace --stats of the headline (overlapped and --sync), C3 and C5 (tools/prof_lines.py)
#   pmc    FETCH_SIZE / WRITE_SIZE, each its own pass, per config (CONFIGS, default "c3 c3vp c5vp"): the sub-lines run
#          alone by tools/prof_lines.py -> profiles/traffic.json via tools/traffic.py
# Stops at the first failure.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6prof
mkdir -p $O
export TMPDIR=/tmp
HEAD="--gpus 1 --warmup 5 --recover-rounds 0 --c5-rounds 0 --sync-rounds 0 --no-c1 --no-cpu-baseline --neg-steps 0 --no-peak-detail --tables-out $O/tables.json"
cd /tmp
run() {  # name limit args...
  local name=$1 lim=$2
  shift 2
  echo "[profile] $name" >&2
  timeout -k 10 $lim rocprofv3 "$@" > $O/$name.log 2>&1 || { echo "$name failed"; tail -20 $O/$name.log; exit 1; }
}
for p in ${PASSES:-trace stats pmc}; do case $p in
trace)
  run trace 300 --kernel-trace --output-format csv -d $O/trace -o run -- python3 $R/bench.py $HEAD --steps 20 --no-kernel-timing
  f=$(find $O/trace -name "*kernel_trace.csv" | head -1)
  python3 - "$f" $O/head_trace.csv <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
keep = ["Kernel_Name", "Queue_Id", "Start_Timestamp", "End_Timestamp", "Grid_Size_X", "Workgroup_Size_X", "VGPR_Count",
        "Accum_VGPR_Count", "LDS_Block_Size", "Scratch_Size"]
with open(sys.argv[2], "w", newline="") as f:
    w = csv.writer(f)
    w.writerow(keep)
    for r in rows:
        w.writerow([r.get(k, "").split("(")[0] if k == "Kernel_Name" else r.get(k, "") for k in keep])
print(len(rows), "dispatches")
PY
  rm -rf $O/trace;;
stats)
  run stats_async 300 --kernel-trace --stats --output-format csv -d $O/stats_async -o run -- python3 $R/bench.py $HEAD --steps 20
  run stats_sync 300 --kernel-trace --stats --output-format csv -d $O/stats_sync -o run -- python3 $R/bench.py $HEAD --sync --steps 10
  for l in c3 c5; do
    run stats_$l 300 --kernel-trace --stats --output-format csv -d $O/stats_$l -o run -- python3 $R/tools/prof_lines.py $l --calls 2
  done
  for d in stats_async stats_sync stats_c3 stats_c5; do
    f=$(find $O/$d -name "*kernel_stats.csv" | head -1); cp "$f" $O/${d}_kernel_stats.csv
    rm -rf $O/$d
  done;;
pmc)
  for cfg in ${CONFIGS:-c3 c3vp c5vp}; do
    for ctr in FETCH_SIZE WRITE_SIZE; do
      echo "[profile] pmc $cfg $ctr" >&2
      case $cfg in
        head) CMD="$R/bench.py $HEAD --sync --steps 1 --warmup 1";;
        c2neg) CMD="$R/bench.py $HEAD --steps 1 --warmup 1 --neg-steps 2";;
        *) CMD="$R/tools/prof_lines.py $cfg";;
      esac
      timeout -s KILL 300 rocprofv3 --pmc $ctr --output-format csv -d $O/pmc_${cfg}_$ctr -o run -- \
        python3 $CMD > $O/pmc_${cfg}_$ctr.log 2>&1 \
        || { echo "pmc $cfg $ctr failed"; tail -5 $O/pmc_${cfg}_$ctr.log; exit 1; }
    done
  done
  cp $R/profiles/traffic.json $O/traffic.json
  python3 $R/tools/traffic.py $O $O/pmc_summary.csv $O/traffic.json > $O/traffic.log 2>&1 || { echo "summary failed"; tail -5 $O/traffic.log; exit 1; }
  rm -rf $O/pmc_*/;;
esac; done
ls -la $O
