#!/bin/bash
# PMC passes over the exponentiation-chain probe (one variant): instruction mix, wave cycles, clock.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/pmc_exp
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd /tmp
timeout -s KILL 60 rocprofv3 -L > $R/gpurun_out/pmc_exp/counters.txt 2>&1 || true
V=${1:-5}
for c in "SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE" "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_SALU"; do
  tag=$(echo $c | cut -d' ' -f1)
  timeout -s KILL 60 rocprofv3 --pmc $c --output-format csv -d $R/gpurun_out/pmc_exp/$tag -o run -- $R/tools/microbench/expchain $V > $R/gpurun_out/pmc_exp/$tag.log 2>&1 || { echo "pmc $c failed"; tail -5 $R/gpurun_out/pmc_exp/$tag.log; }
done
find $R/gpurun_out/pmc_exp -name "*counter_collection.csv" | while read f; do echo "== $f"; python3 - "$f" <<'PY'
import csv,sys,collections
rows=list(csv.DictReader(open(sys.argv[1])))
agg=collections.defaultdict(float)
n=collections.Counter()
for r in rows:
    if 'k_pow' not in r.get('Kernel_Name',''): continue
    agg[(r['Dispatch_Id'],r['Counter_Name'])]+=float(r['Counter_Value'])
last={}
for (d,c),v in agg.items(): last[c]=(d,v)
for c,(d,v) in sorted(last.items()): print(c, d, v)
PY
done
