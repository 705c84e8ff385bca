// Peak-rate probe for the roofline denominator: dependency-free v_mad_u64_u32 streams on every CU
// (8 independent accumulators per lane, 8 waves per CU).  Loaded by bench.py (libdrandprobe.so).
#include <hip/hip_runtime.h>
#include <stdint.h>

constexpr int ITERS = 4096;
constexpr int CH = 8;

__global__ void __launch_bounds__(256) k_probe_mad(uint64_t* out, uint32_t seed) {
  uint32_t a = seed + threadIdx.x, b = seed * 3 + 7;
  uint64_t acc[CH];
  for (int c = 0; c < CH; ++c) acc[c] = c + threadIdx.x;
  for (int i = 0; i < ITERS; ++i) {
#pragma unroll
    for (int c = 0; c < CH; ++c) asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(acc[c]) : "v"(a), "v"(b) : "vcc");
  }
  uint64_t s = 0;
  for (int c = 0; c < CH; ++c) s ^= acc[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

// lane-MACs per second of v_mad_u64_u32 over the whole device; returns 0 on success
extern "C" int probe_mad_rate(int device, double* macs_per_s, int* cus, int* clock_khz) {
  if (hipSetDevice(device) != hipSuccess) return -1;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) != hipSuccess) return -1;
  *cus = prop.multiProcessorCount;
  *clock_khz = prop.clockRate;
  int blocks = prop.multiProcessorCount * 8, threads = 256;
  uint64_t* d;
  if (hipMalloc(&d, sizeof(uint64_t) * blocks * threads) != hipSuccess) return -1;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipLaunchKernelGGL(k_probe_mad, dim3(blocks), dim3(threads), 0, 0, d, 1u);
  hipDeviceSynchronize();
  hipEventRecord(e0, 0);
  for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(k_probe_mad, dim3(blocks), dim3(threads), 0, 0, d, 1u);
  hipEventRecord(e1, 0);
  hipEventSynchronize(e1);
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  *macs_per_s = 5.0 * blocks * threads * (double)ITERS * CH / (ms * 1e-3);
  hipEventDestroy(e0);
  hipEventDestroy(e1);
  hipFree(d);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
