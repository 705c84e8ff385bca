#!/bin/bash
# Round-5 A/B of the cross-round isolation's level shapes: the headline + c2_negative lines only, per DG_XR_QPG value.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for q in ${QPGS:-4 1 16}; do
  DG_XR_QPG=$q timeout -k 10 300 python -u bench.py --steps ${BENCH_STEPS:-10} --recover-rounds 0 --c5-rounds 0 \
    --sync-rounds 0 --no-c1 --no-cpu-baseline --no-peak-detail --neg-steps ${NEG_STEPS:-10} \
    --tables-out gpurun_out/qpg_$q.tables.json > gpurun_out/qpg_$q.json 2> gpurun_out/qpg_$q.err \
    || { echo "bench qpg=$q failed"; tail -20 gpurun_out/qpg_$q.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); n=d['c2_negative']; print('qpg', sys.argv[2], 'head', d['value'], 'neg', n['value'], n['ms_per_step'], n['checks_per_batch'])" gpurun_out/qpg_$q.json $q
done
