#!/bin/bash
# VALU instruction counts of C5's check-pipeline kernels (one rocprofv3 --pmc pass of SQ counters per library):
# the built library and ALT (default drand_amd/ab/libdrandgpu_m0.so) -> gpurun_out/valu/summary.txt
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/valu
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
CTRS="SQ_INSTS_VALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU"
timeout -s KILL 300 rocprofv3 --pmc $CTRS --output-format csv -d $O/new -o run -- python3 $R/tools/prof_lines.py c5 > $O/new.log 2>&1 || { tail -5 $O/new.log; exit 1; }
if [ -f "${ALT:-$R/drand_amd/ab/libdrandgpu_m0.so}" ]; then
DRAND_GPU_LIB=${ALT:-$R/drand_amd/ab/libdrandgpu_m0.so} timeout -s KILL 300 rocprofv3 --pmc $CTRS --output-format csv -d $O/alt -o run -- python3 $R/tools/prof_lines.py c5 > $O/alt.log 2>&1 || { tail -5 $O/alt.log; exit 1; }
fi
python3 - $O > $O/summary.txt <<'PY'
import csv, glob, os, sys, collections
O = sys.argv[1]
for v in ("new", "alt"):
    fs = glob.glob(os.path.join(O, v, "**", "*counter_collection.csv"), recursive=True)
    if not fs:
        continue
    tot = collections.defaultdict(lambda: collections.defaultdict(float))
    n = collections.Counter()
    for r in csv.DictReader(open(fs[0])):
        k = r["Kernel_Name"].split("(")[0]
        tot[k][r["Counter_Name"]] += float(r["Counter_Value"])
        if r["Counter_Name"] == "SQ_WAVES":
            n[k] += 1
    for k in sorted(tot, key=lambda k: -tot[k].get("SQ_INSTS_VALU", 0))[:12]:
        c = tot[k]
        print(v, k, "dispatches", n[k], " ".join("%s=%.4g" % (x, c[x]) for x in sorted(c)))
PY
cat $O/summary.txt
rm -rf $O/new $O/alt
