#!/bin/bash
# Round-5: the negative lines alone (c2_negative: 1% of sigma replaced; vp_negative: VerifyPartial on C5's set),
# with the headline before them.  BENCH_FLAGS adds options.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u bench.py --steps ${BENCH_STEPS:-10} --recover-rounds 0 --sync-rounds 0 --no-c1 \
  --no-cpu-baseline --neg-steps ${NEG_STEPS:-5} --tables-out gpurun_out/neg_tables.json $BENCH_FLAGS \
  > gpurun_out/neg.json 2> gpurun_out/neg.err || { echo "bench failed"; tail -30 gpurun_out/neg.err; exit 1; }
tail -c 6000 gpurun_out/neg.json
