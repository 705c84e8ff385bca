// Exponentiation-chain probe: x^((p-3)/4) per lane (the Fp2 square roots of hash-to-G2 and sigma decode
// are four / two of these), over 200k lanes, for two Montgomery product schedules and several
// waves-per-SIMD bounds.  Prints microseconds per launch and the achieved lane-MAC rate on the
// algorithmic basis of DESIGN.md §4.2 (288 MACs per multiplication, 222 per squaring).
//   V0: product scanning, one 64-bit column accumulator (fp28.h as shipped)
//   V1: separated operand scanning: 27 lazy 64-bit column sums, then 14 reduction rows of 14
//       independent multiply-adds each (short dependency chains, more registers)
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>
#define DG_TU_HOT 1
#include "../../drand_amd/csrc/field.h"
using namespace dg;

template <int V>
DGI void mul_d(const uint32_t (&x)[14], const uint32_t (&y)[14], uint32_t (&r)[14]) {
  if (V == 0) {
    fp28_mont_mul_d(x, y, r);
    return;
  }
  uint64_t t[27];
#pragma unroll
  for (int k = 0; k < 27; ++k) t[k] = 0;
#pragma unroll
  for (int i = 0; i < 14; ++i)
#pragma unroll
    for (int j = 0; j < 14; ++j) t[i + j] += (uint64_t)x[i] * y[j];
#pragma unroll
  for (int i = 0; i < 14; ++i) {
    uint32_t m = ((uint32_t)t[i] * P_INV28) & FP28_MASK;
#pragma unroll
    for (int j = 0; j < 14; ++j) t[i + j] += (uint64_t)m * P28[j];
    if (i < 26) t[i + 1] += t[i] >> 28;
  }
#pragma unroll
  for (int k = 14; k < 26; ++k) {
    r[k - 14] = (uint32_t)t[k] & FP28_MASK;
    t[k + 1] += t[k] >> 28;
  }
  r[12] = (uint32_t)t[26] & FP28_MASK;
  r[13] = (uint32_t)(t[26] >> 28);
}

template <int V>
DGI void sqr_d(const uint32_t (&x)[14], uint32_t (&r)[14]) {
  if (V == 0) {
    fp28_mont_sqr_d(x, r);
    return;
  }
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
    uint32_t m = ((uint32_t)t[i] * P_INV28) & FP28_MASK;
#pragma unroll
    for (int j = 0; j < 14; ++j) t[i + j] += (uint64_t)m * P28[j];
    if (i < 26) t[i + 1] += t[i] >> 28;
  }
#pragma unroll
  for (int k = 14; k < 26; ++k) {
    r[k - 14] = (uint32_t)t[k] & FP28_MASK;
    t[k + 1] += t[k] >> 28;
  }
  r[12] = (uint32_t)t[26] & FP28_MASK;
  r[13] = (uint32_t)(t[26] >> 28);
}

template <int V, int NSTEPS>
DGI void pow_d(uint32_t (&acc)[14], const uint32_t (&x)[14], int first, const int8_t (&steps)[NSTEPS][2]) {
  uint32_t t0[14], t1[14], t2[14], t3[14], x2[14], nxt[14], m[14];
#pragma unroll
  for (int d = 0; d < 14; ++d) t0[d] = x[d];
  sqr_d<V>(t0, x2);
  mul_d<V>(t0, x2, t1);
  mul_d<V>(t1, x2, t2);
  mul_d<V>(t2, x2, t3);
#pragma unroll
  for (int d = 0; d < 14; ++d) acc[d] = first == 0 ? t0[d] : first == 1 ? t1[d] : first == 2 ? t2[d] : t3[d];
  for (int s = 0; s < NSTEPS; ++s) {
    int k = steps[s][0];
    int idx = steps[s][1];
    for (int j = 0; j < k; ++j) {
      sqr_d<V>(acc, nxt);
#pragma unroll
      for (int d = 0; d < 14; ++d) acc[d] = nxt[d];
    }
    if (idx >= 0) {
#pragma unroll
      for (int d = 0; d < 14; ++d) m[d] = idx == 0 ? t0[d] : idx == 1 ? t1[d] : idx == 2 ? t2[d] : t3[d];
      mul_d<V>(acc, m, nxt);
#pragma unroll
      for (int d = 0; d < 14; ++d) acc[d] = nxt[d];
    }
  }
}

// V2: SOS products, width-4 window (8 odd powers), the table indexed by the wave-uniform schedule entry
DGI void pow_w4(uint32_t (&acc)[14], const uint32_t (&x)[14]) {
  uint32_t tab[8][14], x2[14], nxt[14];
#pragma unroll
  for (int d = 0; d < 14; ++d) tab[0][d] = x[d];
  sqr_d<1>(x, x2);
#pragma unroll
  for (int k = 1; k < 8; ++k) mul_d<1>(tab[k - 1], x2, tab[k]);
  const int first = EXP_PM3D4_W4_FIRST;
#pragma unroll
  for (int d = 0; d < 14; ++d) acc[d] = tab[first][d];
  for (int s = 0; s < EXP_PM3D4_W4_NSTEPS; ++s) {
    const int k = EXP_PM3D4_W4_STEPS[s][0];
    const int idx = EXP_PM3D4_W4_STEPS[s][1];
    for (int j = 0; j < k; ++j) {
      sqr_d<1>(acc, nxt);
#pragma unroll
      for (int d = 0; d < 14; ++d) acc[d] = nxt[d];
    }
    if (idx >= 0) {
      uint32_t m[14];
#pragma unroll
      for (int d = 0; d < 14; ++d) m[d] = tab[idx][d];
      mul_d<1>(acc, m, nxt);
#pragma unroll
      for (int d = 0; d < 14; ++d) acc[d] = nxt[d];
    }
  }
}
// V3: as V2, the table selected by a v_cndmask chain
DGI void pow_w4s(uint32_t (&acc)[14], const uint32_t (&x)[14]) {
  uint32_t tab[8][14], x2[14], nxt[14];
#pragma unroll
  for (int d = 0; d < 14; ++d) tab[0][d] = x[d];
  sqr_d<1>(x, x2);
#pragma unroll
  for (int k = 1; k < 8; ++k) mul_d<1>(tab[k - 1], x2, tab[k]);
  const int first = EXP_PM3D4_W4_FIRST;
#pragma unroll
  for (int d = 0; d < 14; ++d) acc[d] = tab[first][d];
  for (int s = 0; s < EXP_PM3D4_W4_NSTEPS; ++s) {
    const int k = EXP_PM3D4_W4_STEPS[s][0];
    const int idx = EXP_PM3D4_W4_STEPS[s][1];
    for (int j = 0; j < k; ++j) {
      sqr_d<1>(acc, nxt);
#pragma unroll
      for (int d = 0; d < 14; ++d) acc[d] = nxt[d];
    }
    if (idx >= 0) {
      uint32_t m[14];
#pragma unroll
      for (int d = 0; d < 14; ++d) {
        uint32_t v = tab[0][d];
#pragma unroll
        for (int q = 1; q < 8; ++q) v = idx == q ? tab[q][d] : v;
        m[d] = v;
      }
      mul_d<1>(acc, m, nxt);
#pragma unroll
      for (int d = 0; d < 14; ++d) acc[d] = nxt[d];
    }
  }
}

template <int V, int W>
__global__ void __launch_bounds__(128, W) k_pow(const uint32_t* in, uint32_t* out, int n, int reps) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t x[14], a[14];
#pragma unroll
  for (int d = 0; d < 14; ++d) x[d] = in[(size_t)d * n + i];
  for (int r = 0; r < reps; ++r) {
    if (V == 2)
      pow_w4(a, x);
    else if (V == 3)
      pow_w4s(a, x);
    else
      pow_d<V>(a, x, EXP_PM3D4_FIRST, EXP_PM3D4_STEPS);
#pragma unroll
    for (int d = 0; d < 14; ++d) x[d] = a[d];
  }
#pragma unroll
  for (int d = 0; d < 14; ++d) out[(size_t)d * n + i] = x[d];
}

#define CHK(x)                                                                \
  do {                                                                        \
    hipError_t e_ = (x);                                                      \
    if (e_ != hipSuccess) {                                                   \
      printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__);       \
      return 1;                                                               \
    }                                                                         \
  } while (0)

int main(int argc, char** argv) {
  const int only = argc > 1 ? atoi(argv[1]) : -1;  // run one variant (profiling)
  const int n = argc > 2 ? atoi(argv[2]) : 200000, reps = argc > 3 ? atoi(argv[3]) : 4;  // items, chains per lane
  int nsq = 1, nmul = 3;
  for (int s = 0; s < EXP_PM3D4_NSTEPS; ++s) {
    nsq += EXP_PM3D4_STEPS[s][0];
    nmul += EXP_PM3D4_STEPS[s][1] >= 0;
  }
  const double macs = (double)nsq * 222 + (double)nmul * 288;
  printf("exp (p-3)/4: %d squarings + %d multiplications = %.0f algorithmic MACs\n", nsq, nmul, macs);
  std::vector<uint32_t> h(14 * (size_t)n);
  uint64_t s = 88172645463325252ull;
  for (size_t k = 0; k < h.size(); ++k) {
    s ^= s << 13;
    s ^= s >> 7;
    s ^= s << 17;
    h[k] = (uint32_t)s & FP28_MASK;
  }
  for (int i = 0; i < n; ++i) h[13 * (size_t)n + i] &= 0xffff;  // < 2^380 < p
  uint32_t *d_in, *d_out;
  CHK(hipMalloc(&d_in, h.size() * 4));
  CHK(hipMalloc(&d_out, h.size() * 4));
  CHK(hipMemcpy(d_in, h.data(), h.size() * 4, hipMemcpyHostToDevice));
  std::vector<uint32_t> ref(h.size()), got(h.size());
  struct K {
    const char* name;
    void (*f)(const uint32_t*, uint32_t*, int, int);
  } ks[] = {{"V0 W1", k_pow<0, 1>}, {"V0 W2", k_pow<0, 2>}, {"V0 W3", k_pow<0, 3>}, {"V0 W4", k_pow<0, 4>},
            {"V1 W1", k_pow<1, 1>}, {"V1 W2", k_pow<1, 2>}, {"V1 W3", k_pow<1, 3>}, {"V1 W4", k_pow<1, 4>},
            {"V2 W1", k_pow<2, 1>}, {"V2 W2", k_pow<2, 2>}, {"V3 W1", k_pow<3, 1>}, {"V3 W2", k_pow<3, 2>}};
  hipEvent_t e0, e1;
  CHK(hipEventCreate(&e0));
  CHK(hipEventCreate(&e1));
  bool first = true;
  int ki = -1;
  for (auto& k : ks) {
    ++ki;
    if (only >= 0 && ki != only) continue;
    hipLaunchKernelGGL(k.f, dim3((n + 127) / 128), dim3(128), 0, 0, d_in, d_out, n, 1);
    CHK(hipDeviceSynchronize());
    CHK(hipEventRecord(e0, 0));
    hipLaunchKernelGGL(k.f, dim3((n + 127) / 128), dim3(128), 0, 0, d_in, d_out, n, reps);
    CHK(hipEventRecord(e1, 0));
    CHK(hipEventSynchronize(e1));
    float ms = 0;
    CHK(hipEventElapsedTime(&ms, e0, e1));
    CHK(hipMemcpy(got.data(), d_out, got.size() * 4, hipMemcpyDeviceToHost));
    // digit forms may differ by p; compare after packing mod p on the host is overkill: both schedules
    // produce a value < 2p from the same inputs, so compare the packed 12-limb values reduced once
    bool same = true;
    if (first) {
      ref = got;
      first = false;
    } else {
      for (int i = 0; i < n && same; ++i) {
        uint32_t a[14], b[14], wa[12], wb[12];
        for (int d = 0; d < 14; ++d) {
          a[d] = ref[(size_t)d * n + i];
          b[d] = got[(size_t)d * n + i];
        }
        fp28_pack(a, wa);
        fp28_pack(b, wb);
        Fp fa, fb;
        for (int l = 0; l < 12; ++l) {
          fa.l[l] = wa[l];
          fb.l[l] = wb[l];
        }
        same = fp_eq(fp_reduce_once(fa), fp_reduce_once(fb));
      }
    }
    double per_launch_us = ms * 1e3 / reps;
    double rate = (double)n * macs / (per_launch_us * 1e-6) / 1e12;
    printf("%-6s n=%d reps=%d  %9.1f us per launch-exponentiation  %6.2f TMAC/s  %s\n", k.name, n, reps, per_launch_us, rate,
           same ? "match" : "MISMATCH");
  }
  return 0;
}
