// Integer / FP64 multiply throughput microbenchmark for gfx950.
// Measures the per-CU issue rate of the instructions a 381-bit Montgomery
// multiply can be built from, to pick the limb representation.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

constexpr int ITERS = 4096;
constexpr int CH = 8;  // independent chains per thread

__global__ void k_mad_u64_u32(uint64_t* out, uint32_t seed) {
  uint32_t a = seed + threadIdx.x, b = seed * 3 + 7;
  uint64_t acc[CH];
  for (int c = 0; c < CH; ++c) acc[c] = c + threadIdx.x;
  for (int i = 0; i < ITERS; ++i) {
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(acc[c]) : "v"(a), "v"(b) : "vcc");
    }
  }
  uint64_t s = 0; for (int c = 0; c < CH; ++c) s ^= acc[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_mul_lo_hi(uint64_t* out, uint32_t seed) {
  uint32_t a = seed + threadIdx.x, b = seed * 3 + 7;
  uint32_t acc[CH];
  for (int c = 0; c < CH; ++c) acc[c] = c + threadIdx.x;
  for (int i = 0; i < ITERS; ++i) {
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(acc[c]) : "v"(b));
    }
  }
  uint64_t s = 0; for (int c = 0; c < CH; ++c) s ^= acc[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s + a;
}

__global__ void k_mul_lo(uint64_t* out, uint32_t seed) {
  uint32_t b = seed * 3 + 7;
  uint32_t acc[CH];
  for (int c = 0; c < CH; ++c) acc[c] = c + threadIdx.x;
  for (int i = 0; i < ITERS; ++i) {
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(acc[c]) : "v"(b));
    }
  }
  uint64_t s = 0; for (int c = 0; c < CH; ++c) s ^= acc[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_mad_u32_u24(uint64_t* out, uint32_t seed) {
  uint32_t b = seed * 3 + 7;
  uint32_t acc[CH];
  for (int c = 0; c < CH; ++c) acc[c] = c + threadIdx.x;
  for (int i = 0; i < ITERS; ++i) {
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      asm volatile("v_mad_u32_u24 %0, %0, %1, %0" : "+v"(acc[c]) : "v"(b));
    }
  }
  uint64_t s = 0; for (int c = 0; c < CH; ++c) s ^= acc[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_add_co(uint64_t* out, uint32_t seed) {
  uint32_t b = seed * 3 + 7;
  uint32_t acc[CH];
  for (int c = 0; c < CH; ++c) acc[c] = c + threadIdx.x;
  for (int i = 0; i < ITERS; ++i) {
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      asm volatile("v_add_co_u32 %0, vcc, %0, %1" : "+v"(acc[c]) : "v"(b) : "vcc");
    }
  }
  uint64_t s = 0; for (int c = 0; c < CH; ++c) s ^= acc[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_addc(uint64_t* out, uint32_t seed) {
  uint32_t b = seed * 3 + 7;
  uint32_t acc[CH];
  for (int c = 0; c < CH; ++c) acc[c] = c + threadIdx.x;
  for (int i = 0; i < ITERS; ++i) {
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      asm volatile("v_addc_co_u32 %0, vcc, %0, %1, vcc" : "+v"(acc[c]) : "v"(b) : "vcc");
    }
  }
  uint64_t s = 0; for (int c = 0; c < CH; ++c) s ^= acc[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_fma_f64(uint64_t* out, uint32_t seed) {
  double b = 1.0000001 + seed * 1e-12;
  double acc[CH];
  for (int c = 0; c < CH; ++c) acc[c] = c + threadIdx.x;
  for (int i = 0; i < ITERS; ++i) {
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      asm volatile("v_fma_f64 %0, %0, %1, %1" : "+v"(acc[c]) : "v"(b));
    }
  }
  double s = 0; for (int c = 0; c < CH; ++c) s += acc[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = (uint64_t)s;
}

__global__ void k_fma_f32(uint64_t* out, uint32_t seed) {
  float b = 1.0000001f + seed * 1e-12f;
  float acc[CH];
  for (int c = 0; c < CH; ++c) acc[c] = c + threadIdx.x;
  for (int i = 0; i < ITERS; ++i) {
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      asm volatile("v_fma_f32 %0, %0, %1, %1" : "+v"(acc[c]) : "v"(b));
    }
  }
  float s = 0; for (int c = 0; c < CH; ++c) s += acc[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = (uint64_t)s;
}

__global__ void k_lshl_add_u64(uint64_t* out, uint32_t seed) {
  uint64_t b = seed * 3 + 7;
  uint64_t acc[CH];
  for (int c = 0; c < CH; ++c) acc[c] = c + threadIdx.x;
  for (int i = 0; i < ITERS; ++i) {
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      asm volatile("v_lshl_add_u64 %0, %0, 0, %1" : "+v"(acc[c]) : "v"(b));
    }
  }
  uint64_t s = 0; for (int c = 0; c < CH; ++c) s ^= acc[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

typedef void (*kfn)(uint64_t*, uint32_t);

int main() {
  hipDeviceProp_t prop; CHK(hipGetDeviceProperties(&prop, 0));
  printf("device %s CUs %d clock %d kHz\n", prop.gcnArchName, prop.multiProcessorCount, prop.clockRate);
  int blocks = prop.multiProcessorCount * 8, threads = 256;
  uint64_t* d; CHK(hipMalloc(&d, sizeof(uint64_t) * blocks * threads));
  struct { const char* name; kfn f; } ks[] = {
    {"v_mad_u64_u32", k_mad_u64_u32}, {"v_mul_hi_u32", k_mul_lo_hi}, {"v_mul_lo_u32", k_mul_lo},
    {"v_mad_u32_u24", k_mad_u32_u24}, {"v_add_co_u32", k_add_co}, {"v_addc_co_u32", k_addc},
    {"v_fma_f64", k_fma_f64}, {"v_fma_f32", k_fma_f32}, {"v_lshl_add_u64", k_lshl_add_u64}};
  hipEvent_t e0, e1; CHK(hipEventCreate(&e0)); CHK(hipEventCreate(&e1));
  for (auto& k : ks) {
    hipLaunchKernelGGL(k.f, dim3(blocks), dim3(threads), 0, 0, d, 1u);
    CHK(hipDeviceSynchronize());
    CHK(hipEventRecord(e0));
    for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(k.f, dim3(blocks), dim3(threads), 0, 0, d, 1u);
    CHK(hipEventRecord(e1)); CHK(hipEventSynchronize(e1));
    float ms; CHK(hipEventElapsedTime(&ms, e0, e1));
    double ops = 5.0 * blocks * threads * (double)ITERS * CH;
    double rate = ops / (ms * 1e-3);
    // cycles per wave-instruction per SIMD at 2.4 GHz: (CUs*4 SIMD * 2.4e9) / (rate/64)
    double cyc = (prop.multiProcessorCount * 4.0 * 2.4e9) / (rate / 64.0);
    printf("%-16s %8.3f Tops/s (lane-ops)  ~%.2f cyc/wave-instr/SIMD @2.4GHz  (%.3f ms)\n", k.name, rate / 1e12, cyc, ms);
  }
  return 0;
}
