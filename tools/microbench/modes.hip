// Code-generation mode probe: latency (1 wave) and throughput (full chip) of G2 Jacobian doubling
// chains and Fp multiplication chains under the DG_FP_CALL / DG_FLAT build modes (field.h).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include "../../drand_amd/csrc/curve.h"
using namespace dg;
struct G2S { Fp2 x, y, z; };

__global__ void __launch_bounds__(128) k_dbl_chain(const G2S* in, G2S* out, int iters) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  G2J p{in[i].x, in[i].y, in[i].z};
  for (int k = 0; k < iters; ++k) p = jac_dbl(p);
  out[i].x = p.x; out[i].y = p.y; out[i].z = p.z;
}
__global__ void __launch_bounds__(128) k_add_chain(const G2S* in, G2S* out, int iters) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  G2J p{in[i].x, in[i].y, in[i].z};
  G2J q = jac_dbl(p);
  for (int k = 0; k < iters; ++k) p = jac_add(p, q);
  out[i].x = p.x; out[i].y = p.y; out[i].z = p.z;
}
__global__ void __launch_bounds__(128) k_mul_chain(const G2S* in, G2S* out, int iters) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  Fp a = in[i].x.c0, b = in[i].x.c1;
  for (int k = 0; k < iters; ++k) a = fp_mul(a, b);
  out[i].x.c0 = a;
}

int main() {
  const int N = 256 * 4 * 64 * 2;
  G2S *d_in, *d_out;
  hipMalloc(&d_in, sizeof(G2S) * N);
  hipMalloc(&d_out, sizeof(G2S) * N);
  hipMemset(d_in, 0x11, sizeof(G2S) * N);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  struct K { const char* name; void (*f)(const G2S*, G2S*, int); int iters; double mpi; } ks[] = {
      {"fp_mul", k_mul_chain, 2000, 1}, {"g2_dbl", k_dbl_chain, 200, 16}, {"g2_add", k_add_chain, 100, 43}};
  for (auto& k : ks) {
    for (int mode = 0; mode < 2; ++mode) {
      int threads = mode == 0 ? 64 : N;
      int blocks = (threads + 127) / 128, bs = threads < 128 ? threads : 128;
      hipLaunchKernelGGL(k.f, dim3(blocks), dim3(bs), 0, 0, d_in, d_out, 2);
      hipDeviceSynchronize();
      hipEventRecord(e0, 0);
      hipLaunchKernelGGL(k.f, dim3(blocks), dim3(bs), 0, 0, d_in, d_out, k.iters);
      hipEventRecord(e1, 0);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      double per = ms * 1e3 / k.iters;  // us per op per lane (latency) or per wave-op
      double mps = (double)threads * k.iters * k.mpi / (ms * 1e-3);
      printf("%s %-7s %s: %.3f ms, %.2f us/op, %.3g Fp-mul-equiv/s\n", MODE_NAME, k.name,
             mode == 0 ? "1 wave " : "full   ", ms, per, mps);
    }
  }
  return 0;
}
