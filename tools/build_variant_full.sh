#!/bin/bash
# A/B build of all three translation units with extra -D flags into tools/variants/libdrandgpu_<name>.so (load with
# DRAND_GPU_LIB=...).  Tooling only.   bash tools/build_variant_full.sh affl2 -DDG_MSM_AFF_L=2
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
name=$1
shift
C=$R/drand_amd/csrc
O=$R/tools/variants
mkdir -p $O
F="--offload-arch=gfx950 -O3 -std=c++17 -Wno-unused-result -fPIC -c"
/opt/rocm/bin/hipcc $F "$@" -o $O/lib_$name.o $C/drand_gpu.hip &
/opt/rocm/bin/hipcc $F -DDG_FLAT=1 "$@" -o $O/hot_$name.o $C/kernels_hot.hip &
/opt/rocm/bin/hipcc $F -DDG_FLAT=1 "$@" -o $O/ver_$name.o $C/kernels_verify.hip &
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $O/libdrandgpu_$name.so $O/lib_$name.o $O/hot_$name.o $O/ver_$name.o
rm -f $O/lib_$name.o $O/hot_$name.o $O/ver_$name.o
echo $O/libdrandgpu_$name.so
