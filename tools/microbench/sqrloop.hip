// Squaring-loop probe (tooling only): why k_exp_pm3d4's squaring loop -- 301 v_mad_u64_u32 of its 424 instructions,
// an ideal ~0.78 of the multiplier's issue rate -- runs at about half of it.  Every lane runs NIT Montgomery
// squarings in the digit form of fp28.h; the kernel variants separate the column sums from the reduction, and
// the waves per SIMD are set by the launch bounds.  Prints SIMD cycles per wave and iteration at the in-kernel
// clock, beside the issue cycles of the static mix (4.45 cycles per quarter-rate instruction, 2.4 otherwise).
//   V0: fp28_sos_sqr_d as shipped        V1: the 105 column products only (then folded back to 14 digits)
//   V2: the 14 reduction rows only        V3: V0 with 32-bit carries (alignbit + add) instead of 64-bit shifts
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#define DG_TU_HOT 1
#include "../../drand_amd/csrc/field.h"
using namespace dg;

template <int V>
__device__ __forceinline__ void step(uint32_t (&x)[14]) {
  uint32_t r[14];
  if (V == 0) {
    fp28_sos_sqr_d(x, r);
  } else if (V == 1) {
    uint64_t t[27];
    uint32_t x2[14];
#pragma unroll
    for (int i = 0; i < 14; ++i) x2[i] = x[i] << 1;
#pragma unroll
    for (int k = 0; k < 27; ++k) t[k] = 0;
#pragma unroll
    for (int i = 0; i < 14; ++i) {
      t[2 * i] += (uint64_t)x[i] * x[i];
#pragma unroll
      for (int j = i + 1; j < 14; ++j) t[i + j] += (uint64_t)x2[i] * x[j];
    }
#pragma unroll
    for (int k = 0; k < 14; ++k) r[k] = ((uint32_t)t[k] ^ (uint32_t)(t[k + 13] >> 28)) & FP28_MASK;
  } else if (V == 2) {
    uint64_t t[27];
#pragma unroll
    for (int k = 0; k < 27; ++k) t[k] = (uint64_t)x[k % 14] << 20 | x[(k + 3) % 14];
    fp28_sos_reduce(t, r);
  } else {
    uint64_t t[27];
    uint32_t x2[14];
#pragma unroll
    for (int i = 0; i < 14; ++i) x2[i] = x[i] << 1;
#pragma unroll
    for (int k = 0; k < 27; ++k) t[k] = 0;
#pragma unroll
    for (int i = 0; i < 14; ++i) {
      t[2 * i] += (uint64_t)x[i] * x[i];
#pragma unroll
      for (int j = i + 1; j < 14; ++j) t[i + j] += (uint64_t)x2[i] * x[j];
    }
#pragma unroll
    for (int i = 0; i < 14; ++i) {
      const uint32_t m = ((uint32_t)t[i] * P_INV28) & FP28_MASK;
#pragma unroll
      for (int j = 0; j < 14; ++j) t[i + j] += (uint64_t)m * P28[j];
      const uint32_t lo = (uint32_t)t[i], hi = (uint32_t)(t[i] >> 32);
      t[i + 1] += (uint32_t)__builtin_amdgcn_alignbit(hi, lo, 28) | 0ull;  // t[i] >> 28 (t[i] < 2^60)
    }
#pragma unroll
    for (int k = 14; k < 26; ++k) {
      r[k - 14] = (uint32_t)t[k] & FP28_MASK;
      const uint32_t lo = (uint32_t)t[k], hi = (uint32_t)(t[k] >> 32);
      t[k + 1] += (uint32_t)__builtin_amdgcn_alignbit(hi, lo, 28);
    }
    r[12] = (uint32_t)t[26] & FP28_MASK;
    r[13] = (uint32_t)(t[26] >> 28);
  }
#pragma unroll
  for (int d = 0; d < 14; ++d) x[d] = r[d];
}

template <int V, int W>
__global__ void __launch_bounds__(64, W) k_loop(uint32_t* io, int nit, unsigned long long* clk) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t x[14];
#pragma unroll
  for (int d = 0; d < 14; ++d) x[d] = (io[i] * (d + 1) + d) & FP28_MASK;
  const unsigned long long c0 = __builtin_readcyclecounter();
  for (int it = 0; it < nit; ++it) step<V>(x);
  const unsigned long long c1 = __builtin_readcyclecounter();
  uint32_t h = 0;
#pragma unroll
  for (int d = 0; d < 14; ++d) h ^= x[d];
  io[i] = h;
  if (threadIdx.x == 0) clk[blockIdx.x] = c1 - c0;
}

template <int V, int W>
double run(uint32_t* io, unsigned long long* clk, int nit, uint32_t nblocks, double* cyc_per_it) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  hipLaunchKernelGGL((k_loop<V, W>), dim3(nblocks), dim3(64), 0, 0, io, nit, clk);  // warm
  hipEventRecord(a, 0);
  hipLaunchKernelGGL((k_loop<V, W>), dim3(nblocks), dim3(64), 0, 0, io, nit, clk);
  hipEventRecord(b, 0);
  hipEventSynchronize(b);
  float ms = 0;
  hipEventElapsedTime(&ms, a, b);
  unsigned long long* h = (unsigned long long*)malloc(8 * nblocks);
  hipMemcpy(h, clk, 8 * nblocks, hipMemcpyDeviceToHost);
  double s = 0;
  for (uint32_t k = 0; k < nblocks; ++k) s += (double)h[k];
  free(h);
  *cyc_per_it = s / nblocks / nit;  // s_memtime-style counter cycles per iteration, one wave
  return ms;
}

int main(int argc, char** argv) {
  const int nit = argc > 1 ? atoi(argv[1]) : 2000;
  hipDeviceProp_t prop;
  hipGetDeviceProperties(&prop, 0);
  const uint32_t cus = prop.multiProcessorCount;
  uint32_t* io;
  unsigned long long* clk;
  const uint32_t maxb = cus * 4 * 8;
  hipMalloc(&io, 64 * maxb * 4);
  hipMalloc(&clk, 8 * maxb);
  hipMemset(io, 1, 64 * maxb * 4);
  double c;
#define RUN(V, W)                                                                                          \
  {                                                                                                        \
    const uint32_t nb = cus * 4 * W;                                                                       \
    double ms = run<V, W>(io, clk, nit, nb, &c);                                                           \
    printf("{\"variant\": %d, \"waves_per_simd\": %d, \"ms\": %.3f, \"wave_cycles_per_iter\": %.1f, "     \
           "\"simd_cycles_per_iter\": %.1f}\n",                                                           \
           V, W, ms, c, ms * 1e-3 * prop.clockRate * 1e3 / ((double)nit * W));                            \
    fflush(stdout);                                                                                        \
  }
  RUN(0, 1) RUN(0, 2) RUN(0, 4) RUN(1, 2) RUN(1, 4) RUN(2, 2) RUN(2, 4) RUN(3, 2) RUN(3, 4)
  return 0;
}
