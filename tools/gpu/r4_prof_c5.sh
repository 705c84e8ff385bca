#!/bin/bash
# rocprofv3 --kernel-trace --stats of the C5 line alone (DRAND_GPU_LIB may select a variant library); the stats CSV and
# a per-kernel summary of the trace (calls, total, mean, min, max us) under gpurun_out/r4prof_c5.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=$GRAFT_REPO_ROOT/gpurun_out/r4prof_c5${TAG:+_$TAG}
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $O/raw -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 1 --warmup 1 --recover-rounds 0 --sync-rounds 0 --no-c1 --no-cpu-baseline --no-peak-detail --no-kernel-timing --tables-out $O/tables.json > $O/bench.log 2>&1 || { echo "profile failed"; tail -20 $O/bench.log; exit 1; }
S=$(find $O/raw -name "*kernel_stats.csv" | head -1)
T=$(find $O/raw -name "*kernel_trace.csv" | head -1)
cp $S $O/kernel_stats.csv
python3 - "$T" > $O/trace_summary.txt <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
d = collections.defaultdict(list)
for r in rows:
    d[r["Kernel_Name"]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
tot = sum(sum(v) for v in d.values())
for k, v in sorted(d.items(), key=lambda kv: -sum(kv[1]))[:40]:
    print("%-28s calls %5d total %10.1f us (%5.1f%%) mean %9.1f min %8.1f max %9.1f" % (k[:28], len(v), sum(v), 100 * sum(v) / tot, sum(v) / len(v), min(v), max(v)))
PY
rm -rf $O/raw
head -45 $O/trace_summary.txt
