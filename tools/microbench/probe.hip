// Peak-rate probe for the roofline denominator (libdrandprobe.so, loaded by bench.py on every rank).
//
// Every lane runs CH = 8 independent v_mad_u64_u32 chains (no data dependency between consecutive
// instructions) on every CU.  Forms (kind):
//   0  carry-out into VCC for every chain (the round-1/2 probe: every instruction writes the same SGPR pair)
//   1  carry-out into a distinct SGPR pair per chain (no shared destination: the rate the kernels can reach)
//   2  the compiler's own form of (uint64_t)a * b + acc (what fp28.h compiles to)
//   3  v_mad_u32_u24 (24-bit operands, 32-bit result: the alternative limb form SURVEY.md §7 asked about)
//   4  v_mul_lo_u32,  5  v_mul_hi_u32 (the two halves of a 32 x 32 -> 64 product done separately)
//   6  v_add_u32, 7 v_fma_f32 (full-rate calibration: the issue rate of the probe's own structure)
//   8  v_fma_f32 on normal floats (7 starts from the integer bit patterns c + lane, f32 denormals: the round-3 3.83-cycle
//      reading of form 7 against the guide's 2 cycles; this form tells whether the denormal operands cost the rate)
//   9  v_fma_f32 with an inline-constant addend (two VGPR sources instead of three: whether the VGPR operand reads,
//      not the multiplier, set the 4-cycle issue of the three-source forms 7, 8 and v_mad_u64_u32)
// Each workgroup stamps s_memtime / s_memrealtime (scalar counter reads) around its loop, so the clock the
// chip held during the measured launches is known (MI355X_MICROARCH.md 'DVFS give-back' item 6): the
// in-kernel clock is the median over workgroups of d(memtime) / d(realtime) x 100 MHz.  The rate is timed
// after at least `warm_s` seconds of back-to-back launches.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <vector>

constexpr int CH = 8;

template <int KIND>
__global__ void __launch_bounds__(256) k_probe(uint64_t* out, uint64_t* clk, uint32_t seed, int iters) {
  uint32_t a = seed + threadIdx.x, b = KIND >= 8 ? __float_as_uint(0.999f) : seed * 3 + 7;
  uint64_t acc[CH];
  uint32_t acc32[CH];
  uint64_t cc[CH];
#pragma unroll
  for (int c = 0; c < CH; ++c) {
    acc[c] = c + threadIdx.x;
    acc32[c] = KIND >= 8 ? __float_as_uint(1.0f + 0.001f * (c + threadIdx.x)) : c + threadIdx.x;
    cc[c] = 0;
  }
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
  const uint64_t r0 = __builtin_amdgcn_s_memrealtime();
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      if (KIND == 0)
        asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(acc[c]) : "v"(a), "v"(b) : "vcc");
      else if (KIND == 1)
        asm volatile("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(acc[c]), "=s"(cc[c]) : "v"(a), "v"(b));
      else if (KIND == 2)
        acc[c] = (uint64_t)a * b + acc[c];
      else if (KIND == 3)
        asm volatile("v_mad_u32_u24 %0, %0, %1, %0" : "+v"(acc32[c]) : "v"(b));
      else if (KIND == 4)
        asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(acc32[c]) : "v"(b));
      else if (KIND == 5)
        asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(acc32[c]) : "v"(b));
      else if (KIND == 6)
        asm volatile("v_add_u32 %0, %0, %1" : "+v"(acc32[c]) : "v"(b));
      else if (KIND == 9)
        asm volatile("v_fma_f32 %0, %0, %1, 1.0" : "+v"(acc32[c]) : "v"(b));
      else
        asm volatile("v_fma_f32 %0, %0, %1, %1" : "+v"(acc32[c]) : "v"(b));
    }
    if (KIND == 2) asm volatile("" : "+v"(a));  // opaque per iteration: the chains cannot be folded into one product
  }
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  const uint64_t r1 = __builtin_amdgcn_s_memrealtime();
  uint64_t s = 0;
#pragma unroll
  for (int c = 0; c < CH; ++c) s ^= acc[c] ^ acc32[c] ^ cc[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (threadIdx.x == 0) {
    clk[2 * blockIdx.x] = t1 - t0;
    clk[2 * blockIdx.x + 1] = r1 - r0;
  }
}

typedef void (*ProbeFn)(uint64_t*, uint64_t*, uint32_t, int);
static ProbeFn probe_fn(int kind) {
  switch (kind) {
    case 0: return k_probe<0>;
    case 1: return k_probe<1>;
    case 2: return k_probe<2>;
    case 3: return k_probe<3>;
    case 4: return k_probe<4>;
    case 5: return k_probe<5>;
    case 6: return k_probe<6>;
    case 8: return k_probe<8>;
    case 9: return k_probe<9>;
    default: return k_probe<7>;
  }
}

// lane-ops per second of form `kind` over the whole device after >= warm_s seconds of launches; the
// in-kernel clock (MHz) of the timed launches; returns 0 on success
extern "C" int probe_run(int device, int kind, double warm_s, double* ops_per_s, double* clock_mhz, int* cus) {
  if (hipSetDevice(device) != hipSuccess) return -1;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) != hipSuccess) return -1;
  *cus = prop.multiProcessorCount;
  const int blocks = prop.multiProcessorCount * 8, threads = 256, iters = 4096;
  uint64_t *d, *clk;
  if (hipMalloc(&d, sizeof(uint64_t) * blocks * threads) != hipSuccess) return -1;
  if (hipMalloc(&clk, sizeof(uint64_t) * 2 * blocks) != hipSuccess) return -1;
  ProbeFn f = probe_fn(kind);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  // warm-up: back-to-back launches for warm_s seconds (the clock settles under load)
  double spent = 0;
  while (spent < warm_s * 1e3) {
    hipEventRecord(e0, 0);
    for (int r = 0; r < 50; ++r) hipLaunchKernelGGL(f, dim3(blocks), dim3(threads), 0, 0, d, clk, 1u, iters);
    hipEventRecord(e1, 0);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    spent += ms;
    if (ms <= 0) break;
  }
  const int reps = 50;
  hipEventRecord(e0, 0);
  for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(f, dim3(blocks), dim3(threads), 0, 0, d, clk, 1u, iters);
  hipEventRecord(e1, 0);
  hipEventSynchronize(e1);
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  *ops_per_s = (double)reps * blocks * threads * (double)iters * CH / (ms * 1e-3);
  std::vector<uint64_t> h(2 * blocks);
  hipMemcpy(h.data(), clk, sizeof(uint64_t) * 2 * blocks, hipMemcpyDeviceToHost);
  std::vector<double> mhz;
  for (int b = 0; b < blocks; ++b)
    if (h[2 * b + 1]) mhz.push_back((double)h[2 * b] / (double)h[2 * b + 1] * 100.0);
  std::sort(mhz.begin(), mhz.end());
  *clock_mhz = mhz.empty() ? 0.0 : mhz[mhz.size() / 2];
  hipEventDestroy(e0);
  hipEventDestroy(e1);
  hipFree(d);
  hipFree(clk);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

// v_mad_u64_u32 lane-MACs per second with distinct carry destinations (kind 1), the round-2 entry point
extern "C" int probe_mad_rate(int device, double* macs_per_s, int* cus, int* clock_khz) {
  double mhz = 0;
  int rc = probe_run(device, 1, 2.0, macs_per_s, &mhz, cus);
  *clock_khz = (int)(mhz * 1e3);
  return rc;
}
