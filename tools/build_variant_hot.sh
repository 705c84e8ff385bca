#!/bin/bash
# A/B build of the hot translation unit (kernels_hot.hip: the phase kernels, the MSMs, Recover's MSM lanes) with extra
# -D flags, linked with the current library, verify and check objects into tools/variants/libdrandgpu_<name>.so (load
# with DRAND_GPU_LIB=...).  Tooling only; run build() first.   bash tools/build_variant_hot.sh sos -DDG_SEQ_SOS=1
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
name=$1
shift
C=$R/drand_amd/csrc
O=$R/tools/variants
mkdir -p $O
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -Wno-unused-result -fPIC -c -DDG_FLAT=1 "$@" -o $O/hot_$name.o $C/kernels_hot.hip
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $O/libdrandgpu_$name.so $C/drand_gpu.o $O/hot_$name.o $C/kernels_verify.o $C/kernels_check_?.o
echo $O/libdrandgpu_$name.so
