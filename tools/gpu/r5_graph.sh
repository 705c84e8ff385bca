#!/bin/bash
# Round-5: beacon batches as HIP graphs -- the GPU tests, then headline + c2_negative with DG_GRAPH=1 / 0.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -v --timeout 300 --timeout-method thread \
    > gpurun_out/graph_pytest.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/graph_pytest.log; exit 1; }
  tail -3 gpurun_out/graph_pytest.log
fi
for g in ${GRAPHS:-1 0}; do
  DG_GRAPH=$g DG_XR_SKIP=${DG_XR_SKIP:-1} DG_BENCH_HOSTPROF=1 timeout -k 10 300 python -u bench.py --steps 20 \
    --recover-rounds 0 --c5-rounds 0 --sync-rounds 0 --no-c1 --no-cpu-baseline --no-peak-detail --no-vp-negative \
    --neg-steps 10 > gpurun_out/graph_$g.json 2> gpurun_out/graph_$g.err \
    || { echo "bench graph=$g failed"; tail -20 gpurun_out/graph_$g.err; exit 1; }
  grep hostprof gpurun_out/graph_$g.err
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); n=d['c2_negative']; print('graph', sys.argv[2], 'head', d['value'], d['ms_per_step'], 'neg', n['value'], n['ms_per_step'])" gpurun_out/graph_$g.json $g
done
