// Workgroup-cooperative arithmetic for the latency-bound tail of a verification batch: the Miller
// loops (with the cofactor clearing of the per-key hash sums), the product of the Miller values and the
// one final exponentiation (A11).  One lane doing this is bound by the latency of ~30k dependent Fp
// multiplications (~1.3 us each on gfx950).  Here a 128-lane workgroup (two waves) evaluates every
// formula as a short sequence of PHASES; a phase is a set of independent Fp multiplications, one per
// lane, whose operands and results live in LDS:
//   - an Fp2 x Fp2 product takes 3 lanes (Karatsuba: a0 b0, a1 b1, (a0+a1)(b0+b1)),
//   - an Fp2 x Fp product takes 2 lanes,
// and the linear glue between phases (additions, doubling, halving, multiplication by small constants)
// runs on lane 0.  The critical path of a GT multiplication becomes one Fp product plus two short
// combination steps; a G2 doubling becomes three Fp products deep, an addition six, a Miller doubling
// step (line, f^2, f * line) four.
//
// GT representation: Fp12 = Fp2[w]/(w^6 - xi), xi = 1 + u, f = sum_k e_k w^k.  With v = w^2 this is the
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
DGI Fp12 fp12_from_w(const Fp12W& w) { return Fp12{Fp6{w.e[0], w.e[2], w.e[4]}, Fp6{w.e[1], w.e[3], w.e[5]}}; }

// x / 2 (Montgomery form is linear, so halving the representative halves the value)
DGI Fp fp_half(const Fp& a) {
  uint32_t mask = 0u - (a.l[0] & 1u);
  Fp s;
  uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < 12; ++i) s.l[i] = addc32(a.l[i], P_LIMBS[i] & mask, c, &c);
  Fp r;
#pragma unroll
  for (int i = 0; i < 11; ++i) r.l[i] = (s.l[i] >> 1) | (s.l[i + 1] << 31);
  r.l[11] = (s.l[11] >> 1) | (c << 31);
  return r;
}
DGI Fp2 fp2_half(const Fp2& a) { return Fp2{fp_half(a.c0), fp_half(a.c1)}; }
DGI Fp2 fp2_triple(const Fp2& a) { return fp2_add(fp2_dbl(a), a); }
// 3 b' c with b' = 4 (1 + u): 12 (1 + u) c
DGI Fp2 fp2_mul_b3(const Fp2& c) {
  Fp2 x = fp2_mul_xi(c);
  Fp2 x4 = fp2_dbl(fp2_dbl(x));
  return fp2_add(fp2_dbl(x4), x4);
}

#if defined(__HIP__)
constexpr int CO_THREADS = 128;

// The per-lane product of a phase.  Out of line by default: a cooperative kernel has dozens of phases, and with
// the ~650-instruction product inlined at each (k_pair_miller_coop: 140k instructions) one Miller step streams
// several hundred KB of code through the 64 KB instruction cache with only two waves to hide the fetches; one
// shared routine stays resident.  DG_COOP_INLINE=1 inlines it (A/B).
#ifndef DG_COOP_INLINE
#define DG_COOP_INLINE 0
#endif
__device__ __forceinline__ Fp co_mul(const Fp& a, const Fp& b) {
#if DG_COOP_INLINE
  return fp_mul_inl(a, b);
#else
  return fp_mul(a, b);
#endif
}

// product jobs: o = a * b
struct CoM2 {
  const Fp2* a;
  const Fp2* b;
  Fp2* o;
};
struct CoM1 {
  const Fp2* a;
  const Fp* b;
  Fp2* o;
};

template <int N>
__device__ __forceinline__ CoM2 co_pick(const CoM2 (&j)[N], int q) {
  CoM2 r = j[0];
#pragma unroll
  for (int k = 1; k < N; ++k)
    if (q == k) r = j[k];
  return r;
}
template <int N>
__device__ __forceinline__ CoM1 co_pick(const CoM1 (&j)[N], int q) {
  CoM1 r = j[0];
#pragma unroll
  for (int k = 1; k < N; ++k)
    if (q == k) r = j[k];
  return r;
}
__device__ __forceinline__ Fp co_kara_operand(const Fp2& a, int m) {
  return m == 0 ? a.c0 : (m == 1 ? a.c1 : fp_add(a.c0, a.c1));
}
__device__ __forceinline__ Fp2 co_kara_combine(const Fp* t) {
  return Fp2{fp_sub(t[0], t[1]), fp_sub(fp_sub(t[2], t[0]), t[1])};
}

// one phase of N2 Fp2 x Fp2 and N1 Fp2 x Fp products (3 N2 + 2 N1 <= 128); tmp: 128 Fp in LDS
template <int N2, int N1>
__device__ __forceinline__ void co_phase(const CoM2 (&j2)[N2], const CoM1 (&j1)[N1], Fp* tmp) {
  static_assert(3 * N2 + 2 * N1 <= CO_THREADS, "phase too wide");
  const int t = threadIdx.x;
  if (t < 3 * N2) {
    int q = t / 3, m = t - 3 * q;
    CoM2 j = co_pick(j2, q);
    tmp[t] = co_mul(co_kara_operand(*j.a, m), co_kara_operand(*j.b, m));
  } else if (t < 3 * N2 + 2 * N1) {
    int u = t - 3 * N2, q = u / 2, m = u - 2 * q;
    CoM1 j = co_pick(j1, q);
    tmp[t] = co_mul(m ? j.a->c1 : j.a->c0, *j.b);
  }
  __syncthreads();
  if (t < 2 * N2) {
    int q = t >> 1, c = t & 1;
    CoM2 j = co_pick(j2, q);
    const Fp* r = tmp + 3 * q;
    if (c == 0)
      j.o->c0 = fp_sub(r[0], r[1]);
    else
      j.o->c1 = fp_sub(fp_sub(r[2], r[0]), r[1]);
  } else if (t < 2 * N2 + N1) {
    int u = t - 2 * N2;
    CoM1 j = co_pick(j1, u);
    *j.o = Fp2{tmp[3 * N2 + 2 * u], tmp[3 * N2 + 2 * u + 1]};
  }
  __syncthreads();
}
template <int N2>
__device__ __forceinline__ void co_phase(const CoM2 (&j2)[N2], Fp* tmp) {
  static_assert(3 * N2 <= CO_THREADS, "phase too wide");
  const int t = threadIdx.x;
  if (t < 3 * N2) {
    int q = t / 3, m = t - 3 * q;
    CoM2 j = co_pick(j2, q);
    tmp[t] = co_mul(co_kara_operand(*j.a, m), co_kara_operand(*j.b, m));
  }
  __syncthreads();
  if (t < 2 * N2) {
    int q = t >> 1, c = t & 1;
    CoM2 j = co_pick(j2, q);
    const Fp* r = tmp + 3 * q;
    if (c == 0)
      j.o->c0 = fp_sub(r[0], r[1]);
    else
      j.o->c1 = fp_sub(fp_sub(r[2], r[0]), r[1]);
  }
  __syncthreads();
}
// Phase with its jobs given as switch-based loaders/storers (lambdas over LDS objects): every operand is
// a constant LDS address in its own branch, so loads are ds_read (a table of job pointers would be
// placed in scratch and dereferenced through flat loads).
template <int N2, int N1, class LD2, class ST2, class LD1, class ST1>
__device__ __forceinline__ void co_phase_f(LD2 ld2, ST2 st2, LD1 ld1, ST1 st1, Fp* tmp) {
  static_assert(3 * N2 + 2 * N1 <= CO_THREADS, "phase too wide");
  const int t = threadIdx.x;
  if (t < 3 * N2) {
    int q = t / 3, m = t - 3 * q;
    Fp2 a, b;
    ld2(q, a, b);
    tmp[t] = co_mul(co_kara_operand(a, m), co_kara_operand(b, m));
  } else if (t < 3 * N2 + 2 * N1) {
    int u = t - 3 * N2, q = u / 2, m = u - 2 * q;
    Fp2 a;
    Fp b;
    ld1(q, a, b);
    tmp[t] = co_mul(m ? a.c1 : a.c0, b);
  }
  __syncthreads();
  if (t < 2 * N2) {
    int q = t >> 1, c = t & 1;
    const Fp* r = tmp + 3 * q;
    st2(q, c, c == 0 ? fp_sub(r[0], r[1]) : fp_sub(fp_sub(r[2], r[0]), r[1]));
  } else if (t < 2 * N2 + N1) {
    int u = t - 2 * N2;
    st1(u, Fp2{tmp[3 * N2 + 2 * u], tmp[3 * N2 + 2 * u + 1]});
  }
  __syncthreads();
}
#define CO_L2(k, A, B) \
  case k:              \
    a_ = *(A);         \
    b_ = *(B);         \
    break;
#define CO_S2(k, O)     \
  case k:               \
    cm((O), c_) = v_;   \
    break;
#define CO_L1(k, A, B) \
  case k:              \
    a_ = *(A);         \
    b_ = *(B);         \
    break;
#define CO_S1(k, O) \
  case k:           \
    *(O) = v_;      \
    break;
#define CO_LD2(...) [&](int q_, Fp2& a_, Fp2& b_) { switch (q_) { __VA_ARGS__ } }
#define CO_ST2(...) [&](int q_, int c_, const Fp& v_) { switch (q_) { __VA_ARGS__ } }
#define CO_LD1(...) [&](int q_, Fp2& a_, Fp& b_) { switch (q_) { __VA_ARGS__ } }
#define CO_ST1(...) [&](int q_, const Fp2& v_) { switch (q_) { __VA_ARGS__ } }
#define CO_NO_LD1 [&](int, Fp2&, Fp&) {}
#define CO_NO_ST1 [&](int, const Fp2&) {}

// Component-parallel glue: lanes 2g + c, g < ngroups, run the body for component c (0: real, 1: u) of
// group g's outputs; the linear Fp2 operations of the formulas are component-wise.
#define CO_LANES(ngroups, ...)                  \
  do {                                          \
    const int t_ = threadIdx.x;                 \
    if (t_ < 2 * (ngroups)) {                   \
      const int c = t_ & 1, g = t_ >> 1;        \
      (void)g;                                  \
      __VA_ARGS__;                              \
    }                                           \
    __syncthreads();                            \
  } while (0)
__device__ __forceinline__ Fp& cm(Fp2* x, int c) { return c ? x->c1 : x->c0; }
__device__ __forceinline__ const Fp& cm(const Fp2* x, int c) { return c ? x->c1 : x->c0; }
__device__ __forceinline__ Fp fp_triple(const Fp& a) { return fp_add(fp_dbl(a), a); }
// lane-0 glue; everyone waits
#define CO_SERIAL(...)      \
  do {                      \
    if (threadIdx.x == 0) { \
      __VA_ARGS__;          \
    }                       \
    __syncthreads();        \
  } while (0)

// ---------------------------------------------------------------- GT arithmetic
struct CoGT {
  Fp ctb[72];   // contributions of the products to the output components
  Fp half[36];  // first summation level
  Fp tmp[CO_THREADS];
  Fp2 gamma[6];  // Frobenius constants xi^(k (p-1) / 6)
};

// GT multiplication in three short steps: (1) the 36 Fp2 products as 108 Fp products (Karatsuba, one
// per lane); (2) 72 lanes turn each product into its contribution to one component of one output
// coefficient, wrapped terms (i + j >= 6) already multiplied by xi; (3) a two-level sum, 36 then 12
// lanes.  At most 3 dependent Fp additions per lane after the products, instead of ~16 on 6 lanes.
//   contribution of a_i b_j = (t0 - t1) + (t2 - t0 - t1) u, times xi = 1 + u when wrapped:
//   comp 0: t0 - t1 (plain), 2 t0 - t2 (wrapped);  comp 1: t2 - t0 - t1 (plain), t2 - 2 t1 (wrapped)
__device__ __forceinline__ Fp co_contrib(const Fp* t, int comp, bool wrap) {
  if (comp == 0) return wrap ? fp_sub(fp_dbl(t[0]), t[2]) : fp_sub(t[0], t[1]);
  return wrap ? fp_sub(t[2], fp_dbl(t[1])) : fp_sub(fp_sub(t[2], t[0]), t[1]);
}
// out coefficient o, component comp: sum of `nterm` contributions ctb[(o * nterm + slot) * 2 + comp]
__device__ __forceinline__ void co_sum_contribs(Fp12W* dst, Fp* ctb, Fp* half, int nterm) {
  const int t = threadIdx.x;
  // level 1 (nterm = 6: 36 lanes add pairs; nterm = 3: 12 lanes add the first two)
  const int npair = nterm / 2;
  if (t < 12 * npair) {
    int o = t / (2 * npair), r = t % (2 * npair), p = r / 2, comp = r % 2;
    half[t] = fp_add(ctb[(o * nterm + 2 * p) * 2 + comp], ctb[(o * nterm + 2 * p + 1) * 2 + comp]);
  }
  __syncthreads();
  if (t < 12) {
    int o = t / 2, comp = t % 2;
    Fp acc = half[(o * npair) * 2 + comp];
    for (int p = 1; p < npair; ++p) acc = fp_add(acc, half[(o * npair + p) * 2 + comp]);
    if (nterm & 1) acc = fp_add(acc, ctb[(o * nterm + nterm - 1) * 2 + comp]);
    if (comp == 0)
      dst->e[o].c0 = acc;
    else
      dst->e[o].c1 = acc;
  }
  __syncthreads();
}

// dst = a * b in GT (dst may alias a or b)
__device__ __forceinline__ void co_fp12_mul(Fp12W* dst, const Fp12W* a, const Fp12W* b, CoGT* s) {
  const int t = threadIdx.x;
  if (t < 108) {
    int q = t / 3, m = t - 3 * q;
    s->tmp[t] = co_mul(co_kara_operand(a->e[q / 6], m), co_kara_operand(b->e[q % 6], m));
  }
  __syncthreads();
  if (t < 72) {
    int q = t / 2, comp = t % 2, i = q / 6, j = q % 6, o = (i + j) % 6;
    s->ctb[(o * 6 + i) * 2 + comp] = co_contrib(s->tmp + 3 * q, comp, i + j >= 6);
  }
  __syncthreads();
  co_sum_contribs(dst, s->ctb, s->half, 6);
}
// dst = a * l for a line l = l0 + l2 w^2 + l3 w^3 (nonzero coefficients in L->e[0], e[2], e[3])
__device__ __forceinline__ void co_fp12_mul_line(Fp12W* dst, const Fp12W* a, const Fp12W* L, CoGT* s) {
  const int t = threadIdx.x;
  if (t < 54) {
    int q = t / 3, m = t - 3 * q;  // q = 3 i + jj, line slot {0, 2, 3}[jj]
    int i = q / 3, jj = q - 3 * i;
    s->tmp[t] = co_mul(co_kara_operand(a->e[i], m), co_kara_operand(L->e[jj == 0 ? 0 : jj + 1], m));
  }
  __syncthreads();
  if (t < 36) {
    int q = t / 2, comp = t % 2, i = q / 3, jj = q % 3;
    int k = i + (jj == 0 ? 0 : jj + 1), o = k % 6;
    s->ctb[(o * 3 + jj) * 2 + comp] = co_contrib(s->tmp + 3 * q, comp, k >= 6);
  }
  __syncthreads();
  co_sum_contribs(dst, s->ctb, s->half, 3);
}
__device__ __forceinline__ void co_fp12_copy(Fp12W* dst, const Fp12W* a) {
  if (threadIdx.x < 6) dst->e[threadIdx.x] = a->e[threadIdx.x];
  __syncthreads();
}
// f^(p^6): negate the odd w-coefficients
__device__ __forceinline__ void co_fp12_conj(Fp12W* dst, const Fp12W* a) {
  const int t = threadIdx.x;
  if (t < 6) dst->e[t] = (t & 1) ? fp2_neg(a->e[t]) : a->e[t];
  __syncthreads();
}
// f^p: e_k -> conj(e_k) * gamma_k
__device__ __forceinline__ void co_fp12_frob(Fp12W* dst, const Fp12W* a, CoGT* s) {
  const int t = threadIdx.x;
  if (t < 18) {
    int q = t / 3, m = t - 3 * q;
    s->tmp[t] = co_mul(co_kara_operand(fp2_conj(a->e[q]), m), co_kara_operand(s->gamma[q], m));
  }
  __syncthreads();
  if (t < 6) dst->e[t] = co_kara_combine(s->tmp + 3 * t);
  __syncthreads();
}
__device__ __forceinline__ void co_gt_init(CoGT* s) {
  CO_SERIAL({
    Fp2 d = fp2_const(FROB_D), g1 = fp2_const(FROB_G1), g2 = fp2_const(FROB_G2);
    s->gamma[0] = fp2_one();
    s->gamma[1] = d;
    s->gamma[2] = g1;
    s->gamma[3] = fp2_mul(d, g1);
    s->gamma[4] = g2;
    s->gamma[5] = fp2_mul(d, g2);
  });
}
// inversion on one lane (once per batch)
__device__ __forceinline__ void co_fp12_inv(Fp12W* dst, const Fp12W* a) {
  CO_SERIAL(*dst = fp12_to_w(fp12_inv(fp12_from_w(*a))));
}
// a^z, z = -Z_ABS (a in the cyclotomic subgroup, so a^-1 = conj(a))
__device__ __forceinline__ void co_fp12_exp_z(Fp12W* dst, const Fp12W* a, Fp12W* acc, CoGT* s) {
  co_fp12_copy(acc, a);
  for (int b = 62; b >= 0; --b) {
    co_fp12_mul(acc, acc, acc, s);
    if ((Z_ABS >> b) & 1) co_fp12_mul(acc, acc, a, s);
  }
  co_fp12_conj(dst, acc);
}

// f <- f^(3 (p^12 - 1) / r), the chain of final_exp_cubed (pairing.h).  scratch: 7 Fp12W.
__device__ __forceinline__ void co_final_exp_cubed(Fp12W* f, Fp12W* sc, CoGT* s) {
  Fp12W *f1 = &sc[0], *f2 = &sc[1], *t0 = &sc[2], *t1 = &sc[3], *x = &sc[4], *y = &sc[5], *acc = &sc[6];
  co_fp12_inv(f1, f);
  co_fp12_conj(f2, f);
  co_fp12_mul(f1, f2, f1, s);  // f^(p^6 - 1)
  co_fp12_frob(f2, f1, s);
  co_fp12_frob(f2, f2, s);
  co_fp12_mul(f2, f2, f1, s);  // ^(p^2 + 1)
  co_fp12_exp_z(t0, f2, acc, s);
  co_fp12_conj(x, f2);
  co_fp12_mul(t0, t0, x, s);  // f2^(z-1)
  co_fp12_exp_z(t1, t0, acc, s);
  co_fp12_conj(x, t0);
  co_fp12_mul(t1, t1, x, s);  // f2^((z-1)^2)
  co_fp12_exp_z(x, t1, acc, s);
  co_fp12_frob(y, t1, s);
  co_fp12_mul(x, x, y, s);  // a = t1^(z+p)
  co_fp12_exp_z(y, x, acc, s);
  co_fp12_exp_z(y, y, acc, s);
  co_fp12_frob(t0, x, s);
  co_fp12_frob(t0, t0, s);
  co_fp12_mul(y, y, t0, s);
  co_fp12_conj(t0, x);
  co_fp12_mul(y, y, t0, s);  // b = a^(z^2 + p^2 - 1)
  co_fp12_mul(t0, f2, f2, s);
  co_fp12_mul(t0, t0, f2, s);  // c = f2^3
  co_fp12_mul(f, y, t0, s);
}

// ---------------------------------------------------------------- G2 (Jacobian) arithmetic
struct CoG2 {
  Fp2 x, y, z;
};
struct CoG2Tmp {
  Fp2 v[16];
  Fp tmp[CO_THREADS];
  uint32_t flag;
};

// P <- 2P (dbl-2009-l, a = 0): three product phases, component-parallel glue
__device__ __forceinline__ void co_g2_dbl(CoG2* P, CoG2Tmp* s) {
  Fp2 *A = &s->v[0], *B = &s->v[1], *YZ = &s->v[2], *E = &s->v[3], *XB = &s->v[4], *C = &s->v[5], *D0 = &s->v[6],
      *F = &s->v[7], *DX = &s->v[8], *Y3 = &s->v[9], *C8 = &s->v[10];
  co_phase_f<3, 0>(CO_LD2(CO_L2(0, &P->x, &P->x) CO_L2(1, &P->y, &P->y) CO_L2(2, &P->y, &P->z)), CO_ST2(CO_S2(0, A) CO_S2(1, B) CO_S2(2, YZ)),
                   CO_NO_LD1, CO_NO_ST1, s->tmp);
  CO_LANES(2, {
    if (g == 0) cm(E, c) = fp_triple(cm(A, c));
    else cm(XB, c) = fp_add(cm(&P->x, c), cm(B, c));
  });
  co_phase_f<3, 0>(CO_LD2(CO_L2(0, B, B) CO_L2(1, XB, XB) CO_L2(2, E, E)), CO_ST2(CO_S2(0, C) CO_S2(1, D0) CO_S2(2, F)),
                   CO_NO_LD1, CO_NO_ST1, s->tmp);
  CO_LANES(3, {
    if (g == 0) {
      Fp D = fp_dbl(fp_sub(fp_sub(cm(D0, c), cm(A, c)), cm(C, c)));
      Fp X3 = fp_sub(cm(F, c), fp_dbl(D));
      cm(DX, c) = fp_sub(D, X3);
      cm(&P->x, c) = X3;
    } else if (g == 1) {
      cm(&P->z, c) = fp_dbl(cm(YZ, c));
    } else {
      cm(C8, c) = fp_dbl(fp_dbl(fp_dbl(cm(C, c))));
    }
  });
  co_phase_f<1, 0>(CO_LD2(CO_L2(0, E, DX)), CO_ST2(CO_S2(0, Y3)),
                   CO_NO_LD1, CO_NO_ST1, s->tmp);
  CO_LANES(1, cm(&P->y, c) = fp_sub(cm(Y3, c), cm(C8, c)));
}

// O <- P + Q (add-2007-bl); exceptional cases (an input at infinity, P = +-Q) are resolved on lane 0.
// O may alias P or Q.
__device__ __forceinline__ void co_g2_add(CoG2* O, const CoG2* P, const CoG2* Q, CoG2Tmp* s) {
  Fp2 *Z1Z1 = &s->v[0], *Z2Z2 = &s->v[1], *ZZ = &s->v[2], *Z12 = &s->v[3], *U1 = &s->v[4], *U2 = &s->v[5],
      *S1a = &s->v[6], *S2a = &s->v[7], *S1 = &s->v[8], *S2 = &s->v[9], *H = &s->v[10], *R = &s->v[11],
      *I = &s->v[12], *R2 = &s->v[13], *J = &s->v[14], *V = &s->v[15];
  CO_SERIAL({
    bool pi = fp2_is_zero(P->z), qi = fp2_is_zero(Q->z);
    s->flag = pi ? 1u : (qi ? 2u : 0u);
    if (pi)
      *O = *Q;
    else if (qi)
      *O = *P;
    *Z12 = fp2_add(P->z, Q->z);
  });
  if (s->flag) return;
  co_phase_f<3, 0>(CO_LD2(CO_L2(0, &P->z, &P->z) CO_L2(1, &Q->z, &Q->z) CO_L2(2, Z12, Z12)), CO_ST2(CO_S2(0, Z1Z1) CO_S2(1, Z2Z2) CO_S2(2, ZZ)),
                   CO_NO_LD1, CO_NO_ST1, s->tmp);
  co_phase_f<4, 0>(CO_LD2(CO_L2(0, &P->x, Z2Z2) CO_L2(1, &Q->x, Z1Z1) CO_L2(2, &P->y, &Q->z) CO_L2(3, &Q->y, &P->z)), CO_ST2(CO_S2(0, U1) CO_S2(1, U2) CO_S2(2, S1a) CO_S2(3, S2a)),
                   CO_NO_LD1, CO_NO_ST1, s->tmp);
  co_phase_f<2, 0>(CO_LD2(CO_L2(0, S1a, Z2Z2) CO_L2(1, S2a, Z1Z1)), CO_ST2(CO_S2(0, S1) CO_S2(1, S2)),
                   CO_NO_LD1, CO_NO_ST1, s->tmp);
  CO_LANES(2, {
    if (g == 0) {
      Fp h = fp_sub(cm(U2, c), cm(U1, c));
      cm(H, c) = h;
      cm(Z12, c) = fp_dbl(h);  // I0 = 2H
    } else {
      cm(R, c) = fp_dbl(fp_sub(cm(S2, c), cm(S1, c)));
    }
  });
  CO_SERIAL({
    s->flag = 0;
    if (fp2_is_zero(*H)) {
      // P = Q: double on this lane (practically never); P = -Q: infinity
      if (fp2_is_zero(*R)) {
        G2J d = jac_dbl(G2J{P->x, P->y, P->z});
        *O = CoG2{d.x, d.y, d.z};
      } else {
        *O = CoG2{fp2_zero(), fp2_zero(), fp2_zero()};
      }
      s->flag = 1;
    }
  });
  if (s->flag) return;
  co_phase_f<2, 0>(CO_LD2(CO_L2(0, Z12, Z12) CO_L2(1, R, R)), CO_ST2(CO_S2(0, I) CO_S2(1, R2)),
                   CO_NO_LD1, CO_NO_ST1, s->tmp);
  co_phase_f<2, 0>(CO_LD2(CO_L2(0, H, I) CO_L2(1, U1, I)), CO_ST2(CO_S2(0, J) CO_S2(1, V)),
                   CO_NO_LD1, CO_NO_ST1, s->tmp);
  CO_LANES(2, {
    if (g == 0) {
      Fp X3 = fp_sub(fp_sub(cm(R2, c), cm(J, c)), fp_dbl(cm(V, c)));
      cm(V, c) = fp_sub(cm(V, c), X3);  // V - X3
      cm(I, c) = X3;
    } else {
      cm(ZZ, c) = fp_sub(fp_sub(cm(ZZ, c), cm(Z1Z1, c)), cm(Z2Z2, c));  // 2 Z1 Z2
    }
  });
  co_phase_f<3, 0>(CO_LD2(CO_L2(0, R, V) CO_L2(1, S1, J) CO_L2(2, ZZ, H)), CO_ST2(CO_S2(0, U1) CO_S2(1, U2) CO_S2(2, Z1Z1)),
                   CO_NO_LD1, CO_NO_ST1, s->tmp);
  CO_LANES(1, {
    cm(&O->x, c) = cm(I, c);
    cm(&O->y, c) = fp_sub(cm(U1, c), fp_dbl(cm(U2, c)));
    cm(&O->z, c) = cm(Z1Z1, c);
  });
}

// psi(P) = (conj(x) cx, conj(y) cy, conj(z)) -- one phase; O may alias P
__device__ __forceinline__ void co_g2_psi(CoG2* O, const CoG2* P, CoG2Tmp* s) {
  Fp2 *cx = &s->v[0], *cy = &s->v[1], *a = &s->v[2], *b = &s->v[3], *ox = &s->v[4], *oy = &s->v[5];
  CO_SERIAL({
    *cx = fp2_const(PSI_CX);
    *cy = fp2_const(PSI_CY);
    *a = fp2_conj(P->x);
    *b = fp2_conj(P->y);
  });
  co_phase_f<2, 0>(CO_LD2(CO_L2(0, a, cx) CO_L2(1, b, cy)), CO_ST2(CO_S2(0, ox) CO_S2(1, oy)),
                   CO_NO_LD1, CO_NO_ST1, s->tmp);
  CO_SERIAL({ *O = CoG2{*ox, *oy, fp2_conj(P->z)}; });
}
// O = [z] P (z = -Z_ABS); O must not alias P
__device__ __forceinline__ void co_g2_mul_z(CoG2* O, const CoG2* P, CoG2Tmp* s) {
  CO_SERIAL(*O = *P);
  for (int b = 62; b >= 0; --b) {
    co_g2_dbl(O, s);
    if ((Z_ABS >> b) & 1) co_g2_add(O, O, P, s);
  }
  CO_SERIAL(O->y = fp2_neg(O->y));
}
// P <- h_eff P = [z^2 - z - 1]P + [z - 1]psi(P) + psi^2(2P)  (as g2_clear_cofactor, curve.h); t: 4 CoG2
// psi(P) == [z]P for one window sum of the batched subgroup check (msm.h), cooperatively; *fail = 1 if not
// (a vector store; several workgroups may write the same 1).  p, zp, pp: LDS points, tmp: LDS scratch.
template <class S>
__device__ __forceinline__ void co_subgroup_check(const S* W, CoG2* p, CoG2* zp, CoG2* pp, CoG2Tmp* tmp,
                                                  uint32_t* fail) {
  CO_SERIAL({ *p = CoG2{W->x, W->y, W->z}; });
  co_g2_mul_z(zp, p, tmp);
  co_g2_psi(pp, p, tmp);
  CO_SERIAL({
    if (!jac_eq(G2J{pp->x, pp->y, pp->z}, G2J{zp->x, zp->y, zp->z})) *fail = 1u;
  });
}

__device__ __forceinline__ void co_g2_clear_cofactor(CoG2* P, CoG2* t, CoG2Tmp* s) {
  CoG2 *t1 = &t[0], *t2 = &t[1], *t3 = &t[2], *p0 = &t[3];
  CO_SERIAL(*p0 = *P);
  co_g2_mul_z(t1, p0, s);  // t1 = [z]P
  co_g2_psi(t2, p0, s);    // t2 = psi(P)
  CO_SERIAL(*t3 = *p0);
  co_g2_dbl(t3, s);
  co_g2_psi(t3, t3, s);
  co_g2_psi(t3, t3, s);  // t3 = psi^2(2P)
  CO_SERIAL(t2->y = fp2_neg(t2->y));
  co_g2_add(t3, t3, t2, s);  // t3 = psi^2(2P) - psi(P)
  CO_SERIAL(t2->y = fp2_neg(t2->y));
  co_g2_add(t2, t1, t2, s);  // t2 = [z]P + psi(P)
  co_g2_mul_z(P, t2, s);     // P = [z]([z]P + psi(P))
  co_g2_add(t3, t3, P, s);
  CO_SERIAL(t1->y = fp2_neg(t1->y));
  co_g2_add(t3, t3, t1, s);
  CO_SERIAL(p0->y = fp2_neg(p0->y));
  co_g2_add(P, t3, p0, s);
}

// ---------------------------------------------------------------- Miller loop
// Line functions of pairing.h (homogeneous projective T, M-twist), split into product phases; the line
// l = c0 + c1 w^2 + c4 w^3 goes to L->e[0], e[2], e[3].
struct CoML {
  CoG2 T;      // projective (X, Y, Z)
  Fp2 qx, qy;  // Q affine
  Fp px, py;   // P affine
  Fp2 v[16];
  Fp tmp[CO_THREADS];
};

__device__ __forceinline__ void co_line_dbl(CoML* m, Fp12W* L) {
  Fp2 *xy = &m->v[0], *b = &m->v[1], *cc = &m->v[2], *j = &m->v[3], *yz2 = &m->v[4], *yz = &m->v[5], *a = &m->v[6],
      *e = &m->v[7], *gg = &m->v[8], *h = &m->v[9], *j3 = &m->v[10], *nh = &m->v[11], *bf = &m->v[12],
      *e2 = &m->v[13], *g2 = &m->v[14];
  CoG2* T = &m->T;
  CO_LANES(1, cm(yz, c) = fp_add(cm(&T->y, c), cm(&T->z, c)));
  co_phase_f<5, 0>(CO_LD2(CO_L2(0, &T->x, &T->y) CO_L2(1, &T->y, &T->y) CO_L2(2, &T->z, &T->z) CO_L2(3, &T->x, &T->x) CO_L2(4, yz, yz)), CO_ST2(CO_S2(0, xy) CO_S2(1, b) CO_S2(2, cc) CO_S2(3, j) CO_S2(4, yz2)),
                   CO_NO_LD1, CO_NO_ST1, m->tmp);
  CO_LANES(4, {
    if (g == 0) {
      // e = 12 (1 + u) c: component 0 of (1 + u) c is c0 - c1, component 1 is c0 + c1
      Fp xc = c ? fp_add(cc->c0, cc->c1) : fp_sub(cc->c0, cc->c1);
      Fp x4 = fp_dbl(fp_dbl(xc));
      Fp ec = fp_add(fp_dbl(x4), x4);
      Fp fc = fp_triple(ec);
      Fp bc = cm(b, c);
      cm(e, c) = ec;
      cm(gg, c) = fp_half(fp_add(bc, fc));
      cm(&L->e[0], c) = fp_sub(ec, bc);
      cm(bf, c) = fp_sub(bc, fc);
    } else if (g == 1) {
      Fp hc = fp_sub(fp_sub(cm(yz2, c), cm(b, c)), cm(cc, c));
      cm(h, c) = hc;
      cm(nh, c) = fp_neg(hc);
    } else if (g == 2) {
      cm(a, c) = fp_half(cm(xy, c));
    } else {
      cm(j3, c) = fp_triple(cm(j, c));
    }
  });
  co_phase_f<4, 2>(CO_LD2(CO_L2(0, e, e) CO_L2(1, a, bf) CO_L2(2, gg, gg) CO_L2(3, b, h)), CO_ST2(CO_S2(0, e2) CO_S2(1, &T->x) CO_S2(2, g2) CO_S2(3, &T->z)),
                   CO_LD1(CO_L1(0, j3, &m->px) CO_L1(1, nh, &m->py)), CO_ST1(CO_S1(0, &L->e[2]) CO_S1(1, &L->e[3])), m->tmp);
  CO_LANES(1, cm(&T->y, c) = fp_sub(cm(g2, c), fp_triple(cm(e2, c))));
}

__device__ __forceinline__ void co_line_add(CoML* m, Fp12W* L) {
  Fp2 *qyz = &m->v[0], *qxz = &m->v[1], *th = &m->v[2], *la = &m->v[3], *nth = &m->v[4], *c = &m->v[5],
      *d = &m->v[6], *tq = &m->v[7], *lq = &m->v[8], *e = &m->v[9], *f = &m->v[10], *gv = &m->v[11], *h = &m->v[12],
      *gh = &m->v[13], *y1 = &m->v[14], *y2 = &m->v[15];
  CoG2* T = &m->T;
  co_phase_f<2, 0>(CO_LD2(CO_L2(0, &m->qy, &T->z) CO_L2(1, &m->qx, &T->z)), CO_ST2(CO_S2(0, qyz) CO_S2(1, qxz)),
                   CO_NO_LD1, CO_NO_ST1, m->tmp);
  CO_LANES(2, {
    if (g == 0) {
      Fp tc = fp_sub(cm(&T->y, c), cm(qyz, c));
      cm(th, c) = tc;
      cm(nth, c) = fp_neg(tc);
    } else {
      cm(la, c) = fp_sub(cm(&T->x, c), cm(qxz, c));
    }
  });
  co_phase_f<4, 2>(CO_LD2(CO_L2(0, th, th) CO_L2(1, la, la) CO_L2(2, th, &m->qx) CO_L2(3, la, &m->qy)), CO_ST2(CO_S2(0, c) CO_S2(1, d) CO_S2(2, tq) CO_S2(3, lq)),
                   CO_LD1(CO_L1(0, nth, &m->px) CO_L1(1, la, &m->py)), CO_ST1(CO_S1(0, &L->e[2]) CO_S1(1, &L->e[3])), m->tmp);
  CO_LANES(1, cm(&L->e[0], c) = fp_sub(cm(tq, c), cm(lq, c)));
  co_phase_f<3, 0>(CO_LD2(CO_L2(0, la, d) CO_L2(1, &T->z, c) CO_L2(2, &T->x, d)), CO_ST2(CO_S2(0, e) CO_S2(1, f) CO_S2(2, gv)),
                   CO_NO_LD1, CO_NO_ST1, m->tmp);
  CO_LANES(1, {
    Fp hc = fp_sub(fp_add(cm(e, c), cm(f, c)), fp_dbl(cm(gv, c)));
    cm(h, c) = hc;
    cm(gh, c) = fp_sub(cm(gv, c), hc);
  });
  co_phase_f<4, 0>(CO_LD2(CO_L2(0, la, h) CO_L2(1, th, gh) CO_L2(2, e, &T->y) CO_L2(3, &T->z, e)), CO_ST2(CO_S2(0, &T->x) CO_S2(1, y1) CO_S2(2, y2) CO_S2(3, qyz)),
                   CO_NO_LD1, CO_NO_ST1, m->tmp);
  CO_LANES(1, {
    cm(&T->y, c) = fp_sub(cm(y1, c), cm(y2, c));
    cm(&T->z, c) = cm(qyz, c);
  });
}

// f = Miller loop of (P, Q), P = (m->px, m->py) and Q = (m->qx, m->qy) affine, neither at infinity
// (z < 0: conjugated at the end).  L: line scratch.
__device__ __forceinline__ void co_miller_loop(Fp12W* f, Fp12W* L, CoML* m, CoGT* s) {
  const int t = threadIdx.x;
  if (t < 6) {
    f->e[t] = t == 0 ? fp2_one() : fp2_zero();
    L->e[t] = fp2_zero();
  }
  CO_SERIAL(m->T = CoG2{m->qx, m->qy, fp2_one()});
  for (int b = 62; b >= 0; --b) {
    co_line_dbl(m, L);
    co_fp12_mul(f, f, f, s);
    co_fp12_mul_line(f, f, L, s);
    if ((Z_ABS >> b) & 1) {
      co_line_add(m, L);
      co_fp12_mul_line(f, f, L, s);
    }
  }
  co_fp12_conj(f, f);
}
#endif

}  // namespace dg
