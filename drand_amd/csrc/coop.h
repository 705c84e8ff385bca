// Wave-cooperative GT (Fp12) arithmetic for the single-batch tail of the verify path: the product of
// the per-key Miller values and the one final exponentiation per RLC batch (A11).  A lone lane doing
// this is latency-bound (~30k dependent Fp multiplications); here one 64-lane wave splits every Fp12
// product into its 36 independent Fp2 products, one per lane, staged through LDS, so the critical path
// of a GT multiplication is one Fp2 product plus a 6-term sum.
//
// Representation: Fp12 = Fp2[w]/(w^6 - xi), xi = 1 + u, f = sum_k e_k w^k.  With v = w^2 this is the
// tower of field.h: (a0 + a1 v + a2 v^2) + (b0 + b1 v + b2 v^2) w = [a0, b0, a1, b1, a2, b2].
#pragma once
#include "pairing.h"

namespace dg {

struct Fp12W {
  Fp2 e[6];
};

DGI Fp12W fp12_to_w(const Fp12& a) {
  Fp12W w;
  w.e[0] = a.c0.c0;
  w.e[1] = a.c1.c0;
  w.e[2] = a.c0.c1;
  w.e[3] = a.c1.c1;
  w.e[4] = a.c0.c2;
  w.e[5] = a.c1.c2;
  return w;
}
DGI Fp12 fp12_from_w(const Fp12W& w) {
  return Fp12{Fp6{w.e[0], w.e[2], w.e[4]}, Fp6{w.e[1], w.e[3], w.e[5]}};
}

#if defined(__HIP__)
// All co_* functions are called by every lane of a 128-lane (two-wave) workgroup; buffers live in LDS.
// `prod` is a 36-entry Fp2 LDS scratch.  dst may alias a or b.
// Products run on lanes [CO_BASE, CO_BASE + 36) -- the second wave of a 128-lane workgroup -- so the
// first wave is free for concurrent work (the Miller loop computes its next line on lane 0 while the
// square of f is in flight: different waves, so truly concurrent, not divergent lanes of one wave).
constexpr int CO_BASE = 64;
__device__ __forceinline__ void co_mul_products(const Fp12W* a, const Fp12W* b, Fp2* prod) {
  const int t = (int)threadIdx.x - CO_BASE;
  if (t >= 0 && t < 36) prod[t] = fp2_mul(a->e[t / 6], b->e[t % 6]);
}
__device__ __forceinline__ void co_mul_sums(Fp12W* dst, const Fp2* prod) {
  const int t = (int)threadIdx.x - CO_BASE;
  if (t >= 0 && t < 6) {
    Fp2 lo = fp2_zero(), hi = fp2_zero();
    for (int i = 0; i < 6; ++i) {
      int j = t - i;
      if (j >= 0)
        lo = fp2_add(lo, prod[i * 6 + j]);
      else
        hi = fp2_add(hi, prod[i * 6 + j + 6]);
    }
    dst->e[t] = fp2_add(lo, fp2_mul_xi(hi));
  }
}
__device__ __forceinline__ void co_mul(Fp12W* dst, const Fp12W* a, const Fp12W* b, Fp2* prod) {
  co_mul_products(a, b, prod);
  __syncthreads();
  co_mul_sums(dst, prod);
  __syncthreads();
}
__device__ __forceinline__ void co_copy(Fp12W* dst, const Fp12W* a) {
  const int t = threadIdx.x;
  if (t < 6) dst->e[t] = a->e[t];
  __syncthreads();
}
// f^(p^6): negate the odd w-coefficients
__device__ __forceinline__ void co_conj(Fp12W* dst, const Fp12W* a) {
  const int t = threadIdx.x;
  if (t < 6) dst->e[t] = (t & 1) ? fp2_neg(a->e[t]) : a->e[t];
  __syncthreads();
}
// f^p: e_k -> conj(e_k) * xi^(k (p-1) / 6)
__device__ __forceinline__ void co_frob(Fp12W* dst, const Fp12W* a) {
  const int t = threadIdx.x;
  if (t < 6) {
    Fp2 g = fp2_one();
    Fp2 d = fp2_const(FROB_D);
    if (t == 1) g = d;
    if (t == 2) g = fp2_const(FROB_G1);
    if (t == 3) g = fp2_mul(d, fp2_const(FROB_G1));
    if (t == 4) g = fp2_const(FROB_G2);
    if (t == 5) g = fp2_mul(d, fp2_const(FROB_G2));
    dst->e[t] = fp2_mul(fp2_conj(a->e[t]), g);
  }
  __syncthreads();
}
// inversion on one lane (once per batch)
__device__ __forceinline__ void co_inv(Fp12W* dst, const Fp12W* a) {
  if (threadIdx.x == 0) *dst = fp12_to_w(fp12_inv(fp12_from_w(*a)));
  __syncthreads();
}
// a^z, z = -Z_ABS (a in the cyclotomic subgroup, so a^-1 = conj(a))
__device__ __forceinline__ void co_exp_z(Fp12W* dst, const Fp12W* a, Fp12W* tmp, Fp2* prod) {
  co_copy(tmp, a);
  for (int b = 62; b >= 0; --b) {
    co_mul(tmp, tmp, tmp, prod);
    if ((Z_ABS >> b) & 1) co_mul(tmp, tmp, a, prod);
  }
  co_conj(dst, tmp);
}

// f^(3 (p^12 - 1) / r), same chain as final_exp_cubed (pairing.h); result in *f.  scratch: 7 Fp12W.
__device__ void co_final_exp_cubed(Fp12W* f, Fp12W* s, Fp2* prod) {
  Fp12W *f1 = &s[0], *f2 = &s[1], *t0 = &s[2], *t1 = &s[3], *x = &s[4], *y = &s[5], *tmp = &s[6];
  co_inv(f1, f);
  co_conj(f2, f);
  co_mul(f1, f2, f1, prod);  // f^(p^6 - 1)
  co_frob(f2, f1);
  co_frob(f2, f2);
  co_mul(f2, f2, f1, prod);  // ^(p^2 + 1)
  co_exp_z(t0, f2, tmp, prod);
  co_conj(x, f2);
  co_mul(t0, t0, x, prod);  // f2^(z-1)
  co_exp_z(t1, t0, tmp, prod);
  co_conj(x, t0);
  co_mul(t1, t1, x, prod);  // f2^((z-1)^2)
  co_exp_z(x, t1, tmp, prod);
  co_frob(y, t1);
  co_mul(x, x, y, prod);  // a = t1^(z+p)
  co_exp_z(y, x, tmp, prod);
  co_exp_z(y, y, tmp, prod);
  co_frob(t0, x);
  co_frob(t0, t0);
  co_mul(y, y, t0, prod);
  co_conj(t0, x);
  co_mul(y, y, t0, prod);  // b = a^(z^2 + p^2 - 1)
  co_mul(t0, f2, f2, prod);
  co_mul(t0, t0, f2, prod);  // c = f2^3
  co_mul(f, y, t0, prod);
}

// Multi-lane Miller loop of one pair (P affine G1, Q affine G2, neither at infinity), z < 0: lane 0
// computes the line functions (the G2 doubling/addition steps), lanes CO_BASE.. fold them into f.
// Result (tower layout) written by the caller from *f.
__device__ void co_miller_loop(Fp12W* f, Fp12W* L, Fp2* prod, const G1A& P, const G2A& Q) {
  const int t = threadIdx.x;
  G2Proj T{Q.x, Q.y, fp2_one()};
  if (t < 6) {
    f->e[t] = t == 0 ? fp2_one() : fp2_zero();
    L->e[t] = fp2_zero();
  }
  __syncthreads();
  Fp2 c0, c1, c4;
  for (int b = 62; b >= 0; --b) {
    co_mul_products(f, f, prod);  // f^2 on lanes CO_BASE..
    if (t == 0) line_dbl(T, c0, c1, c4, P.x, P.y);
    __syncthreads();
    co_mul_sums(f, prod);
    if (t == 0) {
      L->e[0] = c0;
      L->e[2] = c1;
      L->e[3] = c4;
    }
    __syncthreads();
    co_mul_products(f, L, prod);
    bool add = (Z_ABS >> b) & 1;
    if (t == 0 && add) line_add(T, Q.x, Q.y, c0, c1, c4, P.x, P.y);
    __syncthreads();
    co_mul_sums(f, prod);
    __syncthreads();
    if (add) {
      if (t == 0) {
        L->e[0] = c0;
        L->e[2] = c1;
        L->e[3] = c4;
      }
      __syncthreads();
      co_mul(f, f, L, prod);
    }
  }
  co_conj(f, f);
}
#endif

}  // namespace dg
