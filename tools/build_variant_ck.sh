#!/bin/bash
# A/B build of Recover's pairing-check pipeline (checks.h): the five kernels_check_*.hip translation units with extra
# -D flags, linked with the current library, hot and verify objects into tools/variants/libdrandgpu_<name>.so (load
# with DRAND_GPU_LIB=...).  Tooling only; run build() first.   bash tools/build_variant_ck.sh w2 -DDG_CK_WAVES=2
# PARTS=bcd: only those parts get the flags (the others link the built objects)
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
name=$1
shift
C=$R/drand_amd/csrc
O=$R/tools/variants
mkdir -p $O
pids=""
for p in a b c d e; do
  if [[ "${PARTS:-abcde}" != *$p* ]]; then cp $C/kernels_check_$p.o $O/ck_${p}_$name.o; continue; fi
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -Wno-unused-result -fPIC -c -DDG_FLAT=1 "$@" -o $O/ck_${p}_$name.o $C/kernels_check_$p.hip &
  pids="$pids $!"
done
for p in $pids; do wait $p; done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $O/libdrandgpu_$name.so $C/drand_gpu.o $C/kernels_hot.o $C/kernels_verify.o $O/ck_?_$name.o
echo $O/libdrandgpu_$name.so
