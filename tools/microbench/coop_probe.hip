// Latency probe of the cooperative GT phases (coop.h): one 128-lane workgroup runs N dependent
// operations of each kind; prints microseconds per operation.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include "../../drand_amd/csrc/coop.h"
using namespace dg;

template <int MODE>
__global__ void __launch_bounds__(128) k_probe(int iters, Fp12W* out, long long* cyc) {
  __shared__ CoGT gt;
  __shared__ Fp12W F, G;
  __shared__ CoG2Tmp g2t;
  __shared__ CoG2 P;
  const int t = threadIdx.x;
  if (t < 6) {
    F.e[t] = Fp2{fp_small(t + 2), fp_small(3 * t + 1)};
    G.e[t] = Fp2{fp_small(5 * t + 7), fp_small(t + 11)};
  }
  if (t == 0) P = CoG2{fp2_one(), fp2_const(FP2_B_G2), fp2_one()};
  __syncthreads();
  long long c0 = clock64();
  for (int i = 0; i < iters; ++i) {
    if (MODE == 0) co_fp12_mul(&F, &F, &G, &gt);
    if (MODE == 1) {  // products only
      if (t < 108) {
        int q = t / 3, m = t - 3 * q;
        gt.tmp[t] = fp_mul_inl(co_kara_operand(F.e[q / 6], m), co_kara_operand(G.e[q % 6], m));
      }
      __syncthreads();
      if (t < 6) F.e[t].c0 = gt.tmp[t];
      __syncthreads();
    }
    if (MODE == 2) {  // barrier + lane-0 Fp2 add only
      CO_SERIAL(F.e[0] = fp2_add(F.e[0], G.e[0]));
    }
    if (MODE == 3) co_g2_dbl(&P, &g2t);
    if (MODE == 4) {  // one lane: fp_mul chain
      if (t == 0) F.e[0].c0 = fp_mul(F.e[0].c0, G.e[0].c1);
      __syncthreads();
    }
  }
  long long c1 = clock64();
  if (t < 6) out[blockIdx.x].e[t] = F.e[t];
  if (t == 0) cyc[blockIdx.x] = c1 - c0;
}

int main() {
  Fp12W* d;
  long long* c;
  hipMalloc(&d, sizeof(Fp12W) * 4);
  hipMalloc(&c, sizeof(long long) * 4);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const char* names[] = {"co_fp12_mul", "products+barrier", "serial fp2_add+barrier", "co_g2_dbl", "lane0 fp_mul"};
  void (*ks[])(int, Fp12W*, long long*) = {k_probe<0>, k_probe<1>, k_probe<2>, k_probe<3>, k_probe<4>};
  for (int k = 0; k < 5; ++k) {
    int iters = 200;
    hipLaunchKernelGGL(ks[k], dim3(1), dim3(128), 0, 0, 2, d, c);
    hipDeviceSynchronize();
    hipEventRecord(e0, 0);
    hipLaunchKernelGGL(ks[k], dim3(1), dim3(128), 0, 0, iters, d, c);
    hipEventRecord(e1, 0);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    long long cy;
    hipMemcpy(&cy, c, 8, hipMemcpyDeviceToHost);
    printf("%-24s %8.2f us/op   %10.0f clk/op (clock64)\n", names[k], ms * 1e3 / iters, (double)cy / iters);
  }
  return 0;
}
