#!/bin/bash
# A/B build of every translation unit with extra -D flags into tools/variants/libdrandgpu_<name>.so (load with
# DRAND_GPU_LIB=...).  Tooling only.   bash tools/build_variant_full.sh noprio -DDG_PRIO=0
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
name=$1
shift
C=$R/drand_amd/csrc
O=$R/tools/variants
mkdir -p $O
F="--offload-arch=gfx950 -O3 -std=c++17 -Wno-unused-result -fPIC -c"
objs=""
/opt/rocm/bin/hipcc $F "$@" -o $O/lib_$name.o $C/drand_gpu.hip &
/opt/rocm/bin/hipcc $F -DDG_FLAT=1 "$@" -o $O/hot_$name.o $C/kernels_hot.hip &
for p in a b c d e f; do
  /opt/rocm/bin/hipcc $F -DDG_FLAT=1 "$@" -o $O/ck${p}_$name.o $C/kernels_check_$p.hip &
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $O/libdrandgpu_$name.so $O/lib_$name.o $O/hot_$name.o \
  $O/ck[a-f]_$name.o
rm -f $O/lib_$name.o $O/hot_$name.o $O/ck[a-f]_$name.o
echo $O/libdrandgpu_$name.so
