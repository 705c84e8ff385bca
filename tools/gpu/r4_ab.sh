#!/bin/bash
# Round-4 A/B runner: every -m gpu test (unless SKIP_TESTS=1), then the headline, C5 and C3 lines alone for each
# variant in HEAD, C5 and C3 (space-separated NAME or NAME:VAR=VALUE[,VAR=VALUE]; LIB=<name> loads
# tools/variants/libdrandgpu_<name>.so).  Prints each value and the named kernels' average times; stops at the first
# failure.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
if [ -z "$SKIP_TESTS" ]; then
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/pytest_gpu.log 2>&1 || { echo "gpu tests failed"; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
fi
COMMON="--no-c1 --no-cpu-baseline --no-peak-detail"
run() {  # kind name envs flags
  local kind=$1 n=$2 envs=$3 flags=$4 e=""
  for kv in ${envs//,/ }; do
    if [[ $kv == LIB=* ]]; then e="$e DRAND_GPU_LIB=$PWD/tools/variants/libdrandgpu_${kv#LIB=}.so"; else e="$e $kv"; fi
  done
  env $e timeout -k 10 400 python -u bench.py $flags $COMMON --tables-out gpurun_out/${kind}_${n}_tables.json > gpurun_out/${kind}_$n.json 2> gpurun_out/${kind}_$n.err || { echo "$kind $n failed"; tail -30 gpurun_out/${kind}_$n.err; exit 1; }
  python3 tools/gpu/ab_print.py $kind $n
}
for a in $HEAD; do n=${a%%:*}; v=""; [[ "$a" == *:* ]] && v=${a#*:}
  run head $n "$v" "--steps ${HEAD_STEPS:-20} --warmup 2 --recover-rounds 0 --c5-rounds 0 --sync-rounds 0" || exit 1; done
for a in $C5; do n=${a%%:*}; v=""; [[ "$a" == *:* ]] && v=${a#*:}
  run c5 $n "$v" "--steps 2 --warmup 1 --recover-rounds 0 --sync-rounds 0" || exit 1; done
for a in $C3; do n=${a%%:*}; v=""; [[ "$a" == *:* ]] && v=${a#*:}
  run c3 $n "$v" "--steps 3 --warmup 1 --c5-rounds 0 --sync-rounds 0" || exit 1; done
