#!/bin/bash
# rocprofv3 --kernel-trace of the headline alone (10 overlapped steps at the environment's hardware queue count); the
# trace's kernel rows (name, queue, start, end) compressed under gpurun_out/r4trace_head${TAG}.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=$GRAFT_REPO_ROOT/gpurun_out/r4trace_head${TAG:+_$TAG}
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/raw -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 2 --recover-rounds 0 --c5-rounds 0 --sync-rounds 0 --no-c1 --no-cpu-baseline --no-peak-detail --no-kernel-timing --tables-out $O/tables.json > $O/bench.log 2>&1 || { echo "trace failed"; tail -20 $O/bench.log; exit 1; }
T=$(find $O/raw -name "*kernel_trace.csv" | head -1)
python3 - "$T" $O/trace.csv <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
keys = [k for k in ("Kernel_Name", "Queue_Id", "Stream_Id", "Start_Timestamp", "End_Timestamp", "Grid_Size", "Workgroup_Size") if k in rows[0]]
with open(sys.argv[2], "w", newline="") as f:
    w = csv.writer(f)
    w.writerow(keys)
    for r in rows:
        w.writerow([r[k] for k in keys])
print(len(rows), "kernel rows;", list(rows[0].keys()))
PY
rm -rf $O/raw
gzip -f $O/trace.csv
tail -1 $O/bench.log | cut -c1-200
