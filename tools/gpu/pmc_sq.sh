#!/bin/bash
# one PMC pass of SQ counters over a blocking 1-step bench (instruction mix and wait cycles per kernel)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out/pmc_sq
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU --output-format csv -d $R/gpurun_out/pmc_sq -o run -- python3 $R/bench.py --sync --steps 1 --warmup 1 --no-cpu-baseline --recover-rounds 0 --c5-rounds 0 > $R/gpurun_out/pmc_sq/log.txt 2>&1 || { echo "pmc failed"; tail -5 $R/gpurun_out/pmc_sq/log.txt; exit 1; }
python3 - <<'PY'
import csv, collections, glob
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob("/root/repo/gpurun_out/pmc_sq/*counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        if r["Kernel_Name"].startswith("k_"):
            acc[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k in ("k_h2c_uncleared", "k_decode_items", "k_msm_chunks"):
    print(k, {c: "%.4g" % (sum(v) / len(v)) for c, v in acc[k].items()})
PY
