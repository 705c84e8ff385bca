#!/bin/bash
# Round-5 isolation-latency A/B: round-5 GPU tests, then headline + c2_negative per configuration
# (name:env pairs in CONFIGS; env "lib=<file>" loads an A/B build through DRAND_GPU_LIB).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 400 python -u -m pytest tests/test_gpu_round5.py -x -v --timeout 120 --timeout-method thread \
    > gpurun_out/lat_pytest.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/lat_pytest.log; exit 1; }
  tail -3 gpurun_out/lat_pytest.log
fi
for cfg in ${CONFIGS:-base: skip:DG_XR_SKIP=1 q1:DG_XR_QPG=1 noprio:lib=tools/variants/libdrandgpu_noprio.so}; do
  name=${cfg%%:*}; kv=${cfg#*:}; envs=""
  case "$kv" in
    lib=*) envs="DRAND_GPU_LIB=${kv#lib=}";;
    "") envs="";;
    *) envs="${kv//,/ }";;
  esac
  env $envs timeout -k 10 300 python -u bench.py --steps ${BENCH_STEPS:-10} --recover-rounds 0 --c5-rounds 0 \
    --sync-rounds 0 --no-c1 --no-cpu-baseline --no-peak-detail --no-vp-negative --neg-steps ${NEG_STEPS:-10} \
    > gpurun_out/lat_$name.json 2> gpurun_out/lat_$name.err \
    || { echo "bench $name failed"; tail -20 gpurun_out/lat_$name.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); n=d['c2_negative']; print(sys.argv[2], 'head', d['value'], 'neg', n['value'], n['ms_per_step'])" gpurun_out/lat_$name.json $name
done
if [ -n "$TRACE" ]; then
  # kernel timeline of the headline (start/end per dispatch with its queue) for the overlap analysis
  cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/lat_trace -o run -- \
    python3 -u bench.py --steps 10 --recover-rounds 0 --c5-rounds 0 --sync-rounds 0 --no-c1 --no-cpu-baseline \
    --no-peak-detail --no-vp-negative --neg-steps 0 > gpurun_out/lat_trace.json 2> gpurun_out/lat_trace.err \
    || { echo "trace failed"; tail -20 gpurun_out/lat_trace.err; exit 1; }
  find gpurun_out/lat_trace -name "*.csv"
fi
