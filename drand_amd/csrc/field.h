// BLS12-381 field tower for the HIP kernels (gfx950), one field element per lane.
//
// Fp:  12 x 32-bit limbs, Montgomery form (R = 2^392), values kept fully reduced in [0, p).
//      Multiplication scans 14 digits of 28 bits with carry-free 64-bit column sums (fp28.h): one
//      v_mad_u64_u32 per partial product on gfx950.
// Fp2 = Fp[u]/(u^2+1), Fp6 = Fp2[v]/(v^3 - xi), Fp12 = Fp6[w]/(w^2 - v), xi = 1 + u.
//
// This restates the arithmetic of the reference's pairing suite (github.com/drand/bls12-381 v0.2.0,
// selected at key/curve.go:12); the restatement is checked against oracle/ in tests/.
#pragma once
#include <stdint.h>

#if defined(__HIP__)
#include <hip/hip_runtime.h>
#define DGI __host__ __device__ __forceinline__
#define DGN static __host__ __device__ __noinline__
#else
#define DGI static inline
#define DGN static
#endif
// pins a value in a register at this point (an optimisation barrier for the table selects of phases.h)
#if defined(__HIP_DEVICE_COMPILE__)
#define DG_PIN(x) asm volatile("" : "+v"(x))
#else
#define DG_PIN(x) asm volatile("" : "+r"(x))
#endif
// Code-size policy (DESIGN.md §code generation).  DGH marks the mid-level routines (Fp2/Fp6 products,
// exponentiations, curve formulas): out of line by default (DG_FLAT=0), inlined into their kernels with
// DG_FLAT=1.  DGN routines (Fp12 / pairing level) are always out of line.
#ifndef DG_FLAT
#define DG_FLAT 0
#endif
#if DG_FLAT
#define DGH DGI
#else
#define DGH DGN
#endif
// Fp12 / pairing level: out of line.  DG_INLINE12=1 inlines them into their callers, an A/B knob only:
// built that way the per-item pairing kernel took a 24-minute compile and spilled ~19k VGPRs.
#ifndef DG_INLINE12
#define DG_INLINE12 0
#endif
#if DG_INLINE12
#define DG12 DGI
#else
#define DG12 DGN
#endif

#include "bls_constants.h"
#include "fp28.h"

namespace dg {

struct Fp {
  uint32_t l[12];
};
struct Fp2 {
  Fp c0, c1;
};
struct Fp6 {
  Fp2 c0, c1, c2;
};
struct Fp12 {
  Fp6 c0, c1;
};

#if defined(DG_OPCOUNT)
// host-only instrumented build (tools/opcount): counts Montgomery multiplications (squarings included)
extern thread_local uint64_t g_fp_mul_count, g_fp_sqr_count, g_fp_inv_count;
#define DG_COUNT_MUL() (++g_fp_mul_count)
#define DG_COUNT_SQR() (++g_fp_sqr_count)
#define DG_COUNT_INV() (++g_fp_inv_count)
#else
#define DG_COUNT_MUL() ((void)0)
#define DG_COUNT_SQR() ((void)0)
#define DG_COUNT_INV() ((void)0)
#endif

// 32-bit add / subtract with carry.  On the device through clang's carry builtins, which lower to the full-rate
// v_add_co_u32 / v_addc_co_u32 (v_sub_co / v_subb_co) chains with the carry in VCC; the 64-bit form below was
// compiled to 64-bit adds (v_lshl_add_u64) and sign shifts, ~8.4k of them in one Fp12 product of the per-item
// pairing (DG_ADDC_BUILTIN=0 keeps it, A/B).
#ifndef DG_ADDC_BUILTIN
#define DG_ADDC_BUILTIN 1
#endif
#if DG_ADDC_BUILTIN && defined(__HIP_DEVICE_COMPILE__)
DGI uint32_t addc32(uint32_t a, uint32_t b, uint32_t cin, uint32_t* cout) {
  unsigned int co;
  const uint32_t s = __builtin_addc(a, b, cin, &co);
  *cout = co;
  return s;
}
DGI uint32_t subb32(uint32_t a, uint32_t b, uint32_t bin, uint32_t* bout) {
  unsigned int bo;
  const uint32_t d = __builtin_subc(a, b, bin, &bo);
  *bout = bo;
  return d;
}
#else
DGI uint32_t addc32(uint32_t a, uint32_t b, uint32_t cin, uint32_t* cout) {
  uint64_t s = (uint64_t)a + b + cin;
  *cout = (uint32_t)(s >> 32);
  return (uint32_t)s;
}
DGI uint32_t subb32(uint32_t a, uint32_t b, uint32_t bin, uint32_t* bout) {
  uint64_t d = (uint64_t)a - b - bin;
  *bout = (uint32_t)(d >> 63);
  return (uint32_t)d;
}
#endif

DGI Fp fp_const(const uint32_t (&c)[12]) {
  Fp r;
#pragma unroll
  for (int i = 0; i < 12; ++i) r.l[i] = c[i];
  return r;
}
DGI Fp fp_zero() {
  Fp r;
#pragma unroll
  for (int i = 0; i < 12; ++i) r.l[i] = 0;
  return r;
}
DGI Fp fp_one() { return fp_const(FP_ONE); }

DGI bool fp_is_zero(const Fp& a) {
  uint32_t o = 0;
#pragma unroll
  for (int i = 0; i < 12; ++i) o |= a.l[i];
  return o == 0;
}
DGI bool fp_eq(const Fp& a, const Fp& b) {
  uint32_t o = 0;
#pragma unroll
  for (int i = 0; i < 12; ++i) o |= a.l[i] ^ b.l[i];
  return o == 0;
}
// r = c ? b : a
DGI Fp fp_sel(bool c, const Fp& a, const Fp& b) {
  Fp r;
#pragma unroll
  for (int i = 0; i < 12; ++i) r.l[i] = c ? b.l[i] : a.l[i];
  return r;
}

// a - p if a >= p (a < 2^384)
DGI Fp fp_reduce_once(const Fp& a) {
  Fp d;
  uint32_t br = 0;
#pragma unroll
  for (int i = 0; i < 12; ++i) d.l[i] = subb32(a.l[i], P_LIMBS[i], br, &br);
  return fp_sel(br == 0, a, d);
}

DGI Fp fp_add(const Fp& a, const Fp& b) {
  Fp s;
  uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < 12; ++i) s.l[i] = addc32(a.l[i], b.l[i], c, &c);
  return fp_reduce_once(s);
}
DGI Fp fp_dbl(const Fp& a) { return fp_add(a, a); }
DGI Fp fp_sub(const Fp& a, const Fp& b) {
  Fp d;
  uint32_t br = 0;
#pragma unroll
  for (int i = 0; i < 12; ++i) d.l[i] = subb32(a.l[i], b.l[i], br, &br);
  uint32_t mask = 0u - br;
  uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < 12; ++i) d.l[i] = addc32(d.l[i], P_LIMBS[i] & mask, c, &c);
  return d;
}
DGI Fp fp_neg(const Fp& a) {
  // p - a, and 0 -> 0
  Fp d;
  uint32_t br = 0;
#pragma unroll
  for (int i = 0; i < 12; ++i) d.l[i] = subb32(P_LIMBS[i], a.l[i], br, &br);
  return fp_sel(fp_is_zero(a), d, a);
}

// Montgomery multiplication / squaring (fp28.h), then one conditional subtraction.
DGI Fp fp28_mul(const Fp& a, const Fp& b) {
  Fp r;
  fp28_mont_mul(a.l, b.l, r.l);
  return fp_reduce_once(r);
}
DGI Fp fp28_sqr(const Fp& a) {
  Fp r;
  fp28_mont_sqr(a.l, r.l);
  return fp_reduce_once(r);
}
// How device callers reach it (DG_FP_CALL):
//   1  out-of-line, the 24 operand limbs passed as scalar arguments (VGPRs), result returned in VGPRs
//   2  inlined at every call site
// fp_mul_inl / fp_sqr_inl are always inlined: the innermost loops (exponentiation chains, the per-lane
// products of the cooperative phases in coop.h).  Host builds (tests/native, tools/opcount) inline
// everything and count the calls (DG_OPCOUNT).
#ifndef DG_FP_CALL
#define DG_FP_CALL 1
#endif
#if defined(__HIP_DEVICE_COMPILE__)
__device__ __forceinline__ Fp fp_mul_inl(const Fp& a, const Fp& b) { return fp28_mul(a, b); }
__device__ __forceinline__ Fp fp_sqr_inl(const Fp& a) { return fp28_sqr(a); }
#if DG_FP_CALL == 1
#define DG_L12(p) p##0, p##1, p##2, p##3, p##4, p##5, p##6, p##7, p##8, p##9, p##10, p##11
#define DG_P12(p)                                                                                      \
  uint32_t p##0, uint32_t p##1, uint32_t p##2, uint32_t p##3, uint32_t p##4, uint32_t p##5, uint32_t p##6, \
      uint32_t p##7, uint32_t p##8, uint32_t p##9, uint32_t p##10, uint32_t p##11
#define DG_A12(x) x.l[0], x.l[1], x.l[2], x.l[3], x.l[4], x.l[5], x.l[6], x.l[7], x.l[8], x.l[9], x.l[10], x.l[11]
__device__ __noinline__ Fp fp_mul_r(DG_P12(a), DG_P12(b)) {
  const uint32_t a[12] = {DG_L12(a)}, b[12] = {DG_L12(b)};
  Fp r;
  fp28_mont_mul(a, b, r.l);
  return fp_reduce_once(r);
}
__device__ __noinline__ Fp fp_sqr_r(DG_P12(a)) {
  const uint32_t a[12] = {DG_L12(a)};
  Fp r;
  fp28_mont_sqr(a, r.l);
  return fp_reduce_once(r);
}
DGI Fp fp_mul(const Fp& a, const Fp& b) { return fp_mul_r(DG_A12(a), DG_A12(b)); }
DGI Fp fp_sqr(const Fp& a) { return fp_sqr_r(DG_A12(a)); }
#elif DG_FP_CALL == 3
// 3 (kernels_check.hip): inlined and serialised -- the operands are pinned in registers before the product and its
// result after it (empty volatile asms that read and write every limb, kept in program order), so one product's
// temporaries are live at a time whatever the formula above it; no calls, so no call frames in scratch
#define DG_PIN_FP12(f)                                                                                                \
  asm volatile("" : "+v"((f).l[0]), "+v"((f).l[1]), "+v"((f).l[2]), "+v"((f).l[3]), "+v"((f).l[4]), "+v"((f).l[5]), \
               "+v"((f).l[6]), "+v"((f).l[7]), "+v"((f).l[8]), "+v"((f).l[9]), "+v"((f).l[10]), "+v"((f).l[11]))
// The product itself is the separated-operand-scanning form of the exponentiation kernel (fp28.h fp28_sos_*: 27
// independent column sums, then 14 reduction rows of independent multiply-adds) unless DG_FP_SOS=0: its dependency
// chains are a few instructions long, where the single-accumulator column scan of fp28_mont_mul chains every
// multiply-add of a column -- latency a lone wave cannot hide (the pipeline kernels run at 1-2 waves per SIMD).
#ifndef DG_FP_SOS
#define DG_FP_SOS 1
#endif
DGI Fp fp_mul(Fp a, Fp b) {
  DG_PIN_FP12(a);
  DG_PIN_FP12(b);
#if DG_FP_SOS
  uint32_t x[14], y[14], d[14];
  fp28_unpack(a.l, x);
  fp28_unpack(b.l, y);
  fp28_sos_mul_d(x, y, d);
  Fp r;
  fp28_pack(d, r.l);
  r = fp_reduce_once(r);
#else
  Fp r = fp28_mul(a, b);
#endif
  DG_PIN_FP12(r);
  return r;
}
DGI Fp fp_sqr(Fp a) {
  DG_PIN_FP12(a);
#if DG_FP_SOS
  uint32_t x[14], d[14];
  fp28_unpack(a.l, x);
  fp28_sos_sqr_d(x, d);
  Fp r;
  fp28_pack(d, r.l);
  r = fp_reduce_once(r);
#else
  Fp r = fp28_sqr(a);
#endif
  DG_PIN_FP12(r);
  return r;
}
#else
DGI Fp fp_mul(const Fp& a, const Fp& b) { return fp28_mul(a, b); }
DGI Fp fp_sqr(const Fp& a) { return fp28_sqr(a); }
#endif
#else
DGI Fp fp_mul(const Fp& a, const Fp& b) {
  DG_COUNT_MUL();
  return fp28_mul(a, b);
}
DGI Fp fp_sqr(const Fp& a) {
  DG_COUNT_SQR();
  return fp28_sqr(a);
}
DGI Fp fp_mul_inl(const Fp& a, const Fp& b) { return fp_mul(a, b); }
DGI Fp fp_sqr_inl(const Fp& a) { return fp_sqr(a); }
#endif

// plain integer (little-endian limbs) -> Montgomery
DGI Fp fp_to_mont(const Fp& a) { return fp_mul(a, fp_const(FP_R2)); }
DGI Fp fp_from_mont(const Fp& a) {
  Fp one = fp_zero();
  one.l[0] = 1;
  return fp_mul(a, one);
}
DGI Fp fp_small(uint32_t v) {
  Fp a = fp_zero();
  a.l[0] = v;
  return fp_to_mont(a);
}

// The digit-form chain is used in the hot translation unit only (hash-to-G2 -8%, decode -13% per launch).
// Built into the library TU as well (round 1), the overlapped batches ran 3-5x slower although every kernel
// was as fast or faster alone; the likely cause is the queue scratch regrowth of DESIGN.md §5.2 (a library
// kernel's private segment outgrowing the prewarmed one), which dg_init now rules out.
#if DG_TU_HOT
// x^e for a fixed exponent given as a width-3 sliding-window schedule (tools/gen_constants.py).
// The schedule is wave-uniform (scalar loads); the odd-power table is selected with v_cndmask.  The chain
// runs in the radix-2^28 digit form (fp28.h): one unpack of the table, one pack and one conditional
// subtraction at the end instead of per step.
template <int NSTEPS>
DGI Fp fp_pow_sched(const Fp& x, int first, const int8_t (&steps)[NSTEPS][2]) {
  Fp x2 = fp_sqr(x);
  Fp t1f = fp_mul(x, x2);
  Fp t2f = fp_mul(t1f, x2);
  Fp t3f = fp_mul(t2f, x2);
  uint32_t t0[14], t1[14], t2[14], t3[14], acc[14], nxt[14], m[14];
  fp28_unpack(x.l, t0);
  fp28_unpack(t1f.l, t1);
  fp28_unpack(t2f.l, t2);
  fp28_unpack(t3f.l, t3);
#pragma unroll
  for (int d = 0; d < 14; ++d) acc[d] = first == 0 ? t0[d] : first == 1 ? t1[d] : first == 2 ? t2[d] : t3[d];
  for (int s = 0; s < NSTEPS; ++s) {
    int k = steps[s][0];
    int idx = steps[s][1];
    for (int j = 0; j < k; ++j) {
      DG_COUNT_SQR();
      fp28_mont_sqr_d(acc, nxt);
#pragma unroll
      for (int d = 0; d < 14; ++d) acc[d] = nxt[d];
    }
    if (idx >= 0) {
#pragma unroll
      for (int d = 0; d < 14; ++d) m[d] = idx == 0 ? t0[d] : idx == 1 ? t1[d] : idx == 2 ? t2[d] : t3[d];
      DG_COUNT_MUL();
      fp28_mont_mul_d(acc, m, nxt);
#pragma unroll
      for (int d = 0; d < 14; ++d) acc[d] = nxt[d];
    }
  }
  Fp r;
  fp28_pack(acc, r.l);
  return fp_reduce_once(r);
}
#else
// x^e for a fixed exponent given as a width-3 sliding-window schedule (tools/gen_constants.py).
// The schedule is wave-uniform (scalar loads); the odd-power table is selected with v_cndmask.
template <int NSTEPS>
DGI Fp fp_pow_sched(const Fp& x, int first, const int8_t (&steps)[NSTEPS][2]) {
  Fp x2 = fp_sqr(x);
  Fp t0 = x;
  Fp t1 = fp_mul(t0, x2);
  Fp t2 = fp_mul(t1, x2);
  Fp t3 = fp_mul(t2, x2);
  Fp acc = first == 0 ? t0 : first == 1 ? t1 : first == 2 ? t2 : t3;
  for (int s = 0; s < NSTEPS; ++s) {
    int k = steps[s][0];
    int idx = steps[s][1];
    for (int j = 0; j < k; ++j) acc = fp_sqr_inl(acc);
    if (idx >= 0) {
      Fp m = fp_sel(idx == 1, t0, t1);
      m = fp_sel(idx == 2, m, t2);
      m = fp_sel(idx == 3, m, t3);
      acc = fp_mul_inl(acc, m);
    }
  }
  return acc;
}
#endif
// a^(p-2): Fermat inversion (~455 multiplications); kept as the cross-check of fp_inv
DGH Fp fp_inv_fermat(const Fp& a) { return fp_pow_sched(a, EXP_PM2_FIRST, EXP_PM2_STEPS); }

// ---- Bernstein-Yang "safegcd" inversion: constant-time divsteps, 30 per batch, on signed 30-bit
// limbs (the modinv32 organisation of libsecp256k1, restated for the 381-bit p).  37 batches = 1110
// divsteps >= the proven bound (49 * 381 + 57) / 17 = 1102 for 381-bit inputs.  ~35k simple integer
// instructions instead of a 455-multiplication exponentiation; public inputs only (verification).
//
// s30_divsteps / s30_update_de / s30_update_fg / s30_normalize adapt libsecp256k1's src/modinv32_impl.h
// (secp256k1_modinv32_divsteps_30, _update_de_30, _update_fg_30, _normalize_30), which carries this notice:
//   Copyright (c) 2020 Peter Dettman, Pieter Wuille.  Distributed under the MIT software license:
//   Permission is hereby granted, free of charge, to any person obtaining a copy of this software and
//   associated documentation files (the "Software"), to deal in the Software without restriction, including
//   without limitation the rights to use, copy, modify, merge, publish, distribute, sublicense, and/or sell
//   copies of the Software, and to permit persons to whom the Software is furnished to do so, subject to the
//   following conditions: The above copyright notice and this permission notice shall be included in all copies
//   or substantial portions of the Software.  THE SOFTWARE IS PROVIDED "AS IS", WITHOUT WARRANTY OF ANY KIND,
//   EXPRESS OR IMPLIED, INCLUDING BUT NOT LIMITED TO THE WARRANTIES OF MERCHANTABILITY, FITNESS FOR A PARTICULAR
//   PURPOSE AND NONINFRINGEMENT.  IN NO EVENT SHALL THE AUTHORS OR COPYRIGHT HOLDERS BE LIABLE FOR ANY CLAIM,
//   DAMAGES OR OTHER LIABILITY, WHETHER IN AN ACTION OF CONTRACT, TORT OR OTHERWISE, ARISING FROM, OUT OF OR IN
//   CONNECTION WITH THE SOFTWARE OR THE USE OR OTHER DEALINGS IN THE SOFTWARE.
constexpr int S30_N = 13;
struct S30 {
  int32_t v[S30_N];
};
DG_CONST int32_t P30[S30_N] = {1073719979, 670826495, 356515835, 721420204, 821437470, 55215066, 288093811,
                                316751073, 752313463, 517541166, 698659258, 982409209, 1704209};
DG_CONST uint32_t P_INV30 = 0x30003u;  // p^-1 mod 2^30

DGI int32_t s30_divsteps(int32_t zeta, uint32_t f, uint32_t g, int32_t& tu, int32_t& tv, int32_t& tq, int32_t& tr) {
  uint32_t u = 1, v = 0, q = 0, r = 1;
#pragma unroll 6
  for (int i = 0; i < 30; ++i) {
    uint32_t c1 = (uint32_t)(zeta >> 31);
    uint32_t c2 = 0u - (g & 1u);
    uint32_t x = (f ^ c1) - c1, y = (u ^ c1) - c1, z = (v ^ c1) - c1;
    g += x & c2;
    q += y & c2;
    r += z & c2;
    c1 &= c2;
    zeta = (zeta ^ (int32_t)c1) - 1;
    f += g & c1;
    u += q & c1;
    v += r & c1;
    g >>= 1;
    u <<= 1;
    v <<= 1;
  }
  tu = (int32_t)u;
  tv = (int32_t)v;
  tq = (int32_t)q;
  tr = (int32_t)r;
  return zeta;
}
DGI void s30_update_de(S30& d, S30& e, int32_t u, int32_t v, int32_t q, int32_t r) {
  const int32_t M30 = 0x3fffffff;
  int32_t sd = d.v[S30_N - 1] >> 31, se = e.v[S30_N - 1] >> 31;
  int32_t md = (u & sd) + (v & se);
  int32_t me = (q & sd) + (r & se);
  int64_t cd = (int64_t)u * d.v[0] + (int64_t)v * e.v[0];
  int64_t ce = (int64_t)q * d.v[0] + (int64_t)r * e.v[0];
  md -= (int32_t)((P_INV30 * (uint32_t)cd + (uint32_t)md) & (uint32_t)M30);
  me -= (int32_t)((P_INV30 * (uint32_t)ce + (uint32_t)me) & (uint32_t)M30);
  cd += (int64_t)P30[0] * md;
  ce += (int64_t)P30[0] * me;
  cd >>= 30;
  ce >>= 30;
#pragma unroll
  for (int i = 1; i < S30_N; ++i) {
    int32_t di = d.v[i], ei = e.v[i];
    cd += (int64_t)u * di + (int64_t)v * ei + (int64_t)P30[i] * md;
    ce += (int64_t)q * di + (int64_t)r * ei + (int64_t)P30[i] * me;
    d.v[i - 1] = (int32_t)cd & M30;
    cd >>= 30;
    e.v[i - 1] = (int32_t)ce & M30;
    ce >>= 30;
  }
  d.v[S30_N - 1] = (int32_t)cd;
  e.v[S30_N - 1] = (int32_t)ce;
}
DGI void s30_update_fg(S30& f, S30& g, int32_t u, int32_t v, int32_t q, int32_t r) {
  const int32_t M30 = 0x3fffffff;
  int64_t cf = (int64_t)u * f.v[0] + (int64_t)v * g.v[0];
  int64_t cg = (int64_t)q * f.v[0] + (int64_t)r * g.v[0];
  cf >>= 30;
  cg >>= 30;
#pragma unroll
  for (int i = 1; i < S30_N; ++i) {
    int32_t fi = f.v[i], gi = g.v[i];
    cf += (int64_t)u * fi + (int64_t)v * gi;
    cg += (int64_t)q * fi + (int64_t)r * gi;
    f.v[i - 1] = (int32_t)cf & M30;
    cf >>= 30;
    g.v[i - 1] = (int32_t)cg & M30;
    cg >>= 30;
  }
  f.v[S30_N - 1] = (int32_t)cf;
  g.v[S30_N - 1] = (int32_t)cg;
}
// d in (-2p, p) -> [0, p), negated first when sign < 0
DGI void s30_normalize(S30& d, int32_t sign) {
  const int32_t M30 = 0x3fffffff;
  int32_t add = d.v[S30_N - 1] >> 31, neg = sign >> 31;
#pragma unroll
  for (int i = 0; i < S30_N; ++i) d.v[i] = ((d.v[i] + (P30[i] & add)) ^ neg) - neg;
#pragma unroll
  for (int i = 0; i < S30_N - 1; ++i) {
    d.v[i + 1] += d.v[i] >> 30;
    d.v[i] &= M30;
  }
  add = d.v[S30_N - 1] >> 31;
#pragma unroll
  for (int i = 0; i < S30_N; ++i) d.v[i] += P30[i] & add;
#pragma unroll
  for (int i = 0; i < S30_N - 1; ++i) {
    d.v[i + 1] += d.v[i] >> 30;
    d.v[i] &= M30;
  }
}
DGI S30 s30_from_fp(const Fp& a) {
  S30 r;
#pragma unroll
  for (int i = 0; i < S30_N; ++i) {
    int bit = 30 * i, w = bit >> 5, sh = bit & 31;
    uint64_t x = (uint64_t)a.l[w] | ((uint64_t)(w + 1 < 12 ? a.l[w + 1] : 0u) << 32);
    r.v[i] = (int32_t)((x >> sh) & 0x3fffffffu);
  }
  return r;
}
DGI Fp s30_to_fp(const S30& d) {
  Fp r;
#pragma unroll
  for (int w = 0; w < 12; ++w) {
    int bit = 32 * w, i = bit / 30, sh = bit - 30 * i;
    uint64_t x = (uint64_t)(uint32_t)d.v[i] | ((uint64_t)(uint32_t)(i + 1 < S30_N ? d.v[i + 1] : 0) << 30);
    if (i + 2 < S30_N) x |= (uint64_t)(uint32_t)d.v[i + 2] << 60;
    r.l[w] = (uint32_t)(x >> sh);
  }
  return r;
}
// Montgomery in, Montgomery out: the plain integer A = a R is inverted, then A^-1 * R^3 * R^-1 = a^-1 R
DGH Fp fp_inv(const Fp& a) {
  DG_COUNT_INV();
  S30 d, e, f, g;
#pragma unroll
  for (int i = 0; i < S30_N; ++i) {
    d.v[i] = 0;
    e.v[i] = 0;
    f.v[i] = P30[i];
  }
  e.v[0] = 1;
  g = s30_from_fp(a);
  int32_t zeta = -1;
  for (int it = 0; it < 37; ++it) {
    int32_t u, v, q, r;
    zeta = s30_divsteps(zeta, (uint32_t)f.v[0], (uint32_t)g.v[0], u, v, q, r);
    s30_update_de(d, e, u, v, q, r);
    s30_update_fg(f, g, u, v, q, r);
  }
  s30_normalize(d, f.v[S30_N - 1]);
  return fp_mul(s30_to_fp(d), fp_const(FP_R3));
}
// returns x^((p-3)/4)
DGH Fp fp_pow_pm3d4(const Fp& a) { return fp_pow_sched(a, EXP_PM3D4_FIRST, EXP_PM3D4_STEPS); }
// sqrt(a) if a is a square (r^2 == a checked by the caller or via return)
DGI bool fp_sqrt(Fp& r, const Fp& a) {
  Fp t = fp_pow_pm3d4(a);
  Fp s = fp_mul(t, a);  // a^((p+1)/4)
  r = s;
  return fp_eq(fp_sqr(s), a);
}

// compare plain (non-Montgomery) value against (p-1)/2: returns a > (p-1)/2
DGI bool fp_plain_gt_half(const Fp& a) {
  uint32_t br = 0;
#pragma unroll
  for (int i = 0; i < 12; ++i) (void)subb32(FP_HALF_PM1[i], a.l[i], br, &br);
  return br != 0;
}
DGI bool fp_lex_largest(const Fp& a) { return fp_plain_gt_half(fp_from_mont(a)); }
DGI uint32_t fp_parity(const Fp& a) { return fp_from_mont(a).l[0] & 1u; }

// big-endian 48 B (top 3 bits of byte 0 masked by caller) -> limbs; returns false if >= p
DGI bool fp_from_be48_plain(Fp& r, const uint8_t* b) {
#pragma unroll
  for (int i = 0; i < 12; ++i) {
    const uint8_t* q = b + 44 - 4 * i;
    r.l[i] = (uint32_t)q[0] << 24 | (uint32_t)q[1] << 16 | (uint32_t)q[2] << 8 | q[3];
  }
  uint32_t br = 0;
#pragma unroll
  for (int i = 0; i < 12; ++i) (void)subb32(r.l[i], P_LIMBS[i], br, &br);
  return br != 0;
}
DGI void fp_to_be48(uint8_t* b, const Fp& a) {
  Fp x = fp_from_mont(a);
#pragma unroll
  for (int i = 0; i < 12; ++i) {
    uint8_t* q = b + 44 - 4 * i;
    q[0] = (uint8_t)(x.l[i] >> 24);
    q[1] = (uint8_t)(x.l[i] >> 16);
    q[2] = (uint8_t)(x.l[i] >> 8);
    q[3] = (uint8_t)x.l[i];
  }
}
// 64 B big-endian (hash_to_field, RFC 9380 §5.2, L = 64) -> Fp: hi * 2^256 + lo mod p
DGI Fp fp_from_be64(const uint8_t* b) {
  Fp hi = fp_zero(), lo = fp_zero();
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const uint8_t* q = b + 28 - 4 * i;
    hi.l[i] = (uint32_t)q[0] << 24 | (uint32_t)q[1] << 16 | (uint32_t)q[2] << 8 | q[3];
    const uint8_t* w = b + 60 - 4 * i;
    lo.l[i] = (uint32_t)w[0] << 24 | (uint32_t)w[1] << 16 | (uint32_t)w[2] << 8 | w[3];
  }
  // values < 2^256 < p: to Montgomery, then hi * (2^256 in Montgomery)
  return fp_add(fp_mul(fp_to_mont(hi), fp_const(FP_2POW256)), fp_to_mont(lo));
}

// ------------------------------------------------------------------------------------------- Fp2
DGI Fp2 fp2_const(const uint32_t (&c)[2][12]) {
  Fp2 r;
#pragma unroll
  for (int i = 0; i < 12; ++i) {
    r.c0.l[i] = c[0][i];
    r.c1.l[i] = c[1][i];
  }
  return r;
}
DGI Fp2 fp2_zero() { return Fp2{fp_zero(), fp_zero()}; }
DGI Fp2 fp2_one() { return Fp2{fp_one(), fp_zero()}; }
DGI bool fp2_is_zero(const Fp2& a) { return fp_is_zero(a.c0) && fp_is_zero(a.c1); }
DGI bool fp2_eq(const Fp2& a, const Fp2& b) { return fp_eq(a.c0, b.c0) && fp_eq(a.c1, b.c1); }
DGI Fp2 fp2_sel(bool c, const Fp2& a, const Fp2& b) { return Fp2{fp_sel(c, a.c0, b.c0), fp_sel(c, a.c1, b.c1)}; }
// DG_FP2_ILV=1 (the pipeline TUs, kernels_check_*.hip): the two coefficients' carry chains interleaved limb by limb.
// A carry chain alone puts a wait state (s_nop) between every two limbs on gfx950 -- a VALU that writes the carry
// (VCC / an SGPR pair) and the next VALU that reads it -- about 11% of the per-item pairing kernels' instructions;
// with the c0 and c1 chains alternating, each carry is read two instructions after it is written.
#ifndef DG_FP2_ILV
#define DG_FP2_ILV 0
#endif
#if DG_FP2_ILV
DGI Fp2 fp2_reduce2(const Fp2& s) {
  Fp2 d;
  uint32_t b0 = 0, b1 = 0;
#pragma unroll
  for (int i = 0; i < 12; ++i) {
    d.c0.l[i] = subb32(s.c0.l[i], P_LIMBS[i], b0, &b0);
    d.c1.l[i] = subb32(s.c1.l[i], P_LIMBS[i], b1, &b1);
  }
  return Fp2{fp_sel(b0 == 0, s.c0, d.c0), fp_sel(b1 == 0, s.c1, d.c1)};
}
DGI Fp2 fp2_add(const Fp2& a, const Fp2& b) {
  Fp2 s;
  uint32_t c0 = 0, c1 = 0;
#pragma unroll
  for (int i = 0; i < 12; ++i) {
    s.c0.l[i] = addc32(a.c0.l[i], b.c0.l[i], c0, &c0);
    s.c1.l[i] = addc32(a.c1.l[i], b.c1.l[i], c1, &c1);
  }
  return fp2_reduce2(s);
}
DGI Fp2 fp2_sub(const Fp2& a, const Fp2& b) {
  Fp2 d;
  uint32_t b0 = 0, b1 = 0;
#pragma unroll
  for (int i = 0; i < 12; ++i) {
    d.c0.l[i] = subb32(a.c0.l[i], b.c0.l[i], b0, &b0);
    d.c1.l[i] = subb32(a.c1.l[i], b.c1.l[i], b1, &b1);
  }
  const uint32_t m0 = 0u - b0, m1 = 0u - b1;
  uint32_t c0 = 0, c1 = 0;
#pragma unroll
  for (int i = 0; i < 12; ++i) {
    d.c0.l[i] = addc32(d.c0.l[i], P_LIMBS[i] & m0, c0, &c0);
    d.c1.l[i] = addc32(d.c1.l[i], P_LIMBS[i] & m1, c1, &c1);
  }
  return d;
}
DGI Fp2 fp2_dbl(const Fp2& a) { return fp2_add(a, a); }
#else
DGI Fp2 fp2_add(const Fp2& a, const Fp2& b) { return Fp2{fp_add(a.c0, b.c0), fp_add(a.c1, b.c1)}; }
DGI Fp2 fp2_sub(const Fp2& a, const Fp2& b) { return Fp2{fp_sub(a.c0, b.c0), fp_sub(a.c1, b.c1)}; }
DGI Fp2 fp2_dbl(const Fp2& a) { return Fp2{fp_dbl(a.c0), fp_dbl(a.c1)}; }
#endif
DGI Fp2 fp2_neg(const Fp2& a) { return Fp2{fp_neg(a.c0), fp_neg(a.c1)}; }
DGI Fp2 fp2_conj(const Fp2& a) { return Fp2{a.c0, fp_neg(a.c1)}; }
// DG_FP2_CALL=1 (the per-item pairing TU): fp2_mul / fp2_sqr are one out-of-line call each (fp2_mul_r below,
// operands and result in VGPRs, the Karatsuba products inlined in the callee) instead of three / two Fp-level calls
#ifndef DG_FP2_CALL
#define DG_FP2_CALL 0
#endif
#if DG_FP2_CALL && defined(__HIP_DEVICE_COMPILE__) && DG_FP_CALL == 1
__device__ __noinline__ Fp2 fp2_mul_r(DG_P12(a), DG_P12(b), DG_P12(c), DG_P12(d));
__device__ __noinline__ Fp2 fp2_sqr_r(DG_P12(a), DG_P12(b));
DGI Fp2 fp2_mul(const Fp2& a, const Fp2& b) { return fp2_mul_r(DG_A12(a.c0), DG_A12(a.c1), DG_A12(b.c0), DG_A12(b.c1)); }
DGI Fp2 fp2_sqr(const Fp2& a) { return fp2_sqr_r(DG_A12(a.c0), DG_A12(a.c1)); }
#else
// DG_FP_PIN2=1 (with DG_FP_CALL=3; the one-wave pipeline kernels): the pins at the Fp2 level instead -- operands
// pinned before the Karatsuba triple, results after -- so its three independent Fp products may interleave (three
// times the independent work per wave, where the 512-entry register file has room for it)
#ifndef DG_FP_PIN2
#define DG_FP_PIN2 0
#endif
#if DG_FP_PIN2 && DG_FP_CALL == 3 && defined(__HIP_DEVICE_COMPILE__)
DGI Fp fp_mul_np(const Fp& a, const Fp& b) {
  uint32_t x[14], y[14], d[14];
  fp28_unpack(a.l, x);
  fp28_unpack(b.l, y);
  fp28_sos_mul_d(x, y, d);
  Fp r;
  fp28_pack(d, r.l);
  return fp_reduce_once(r);
}
#define DG_FP2_PINNED 1
#else
#define DG_FP2_PINNED 0
#endif
// The Karatsuba triple with each operand unpacked to digit form once (fp28.h) and the two sums a0 + a1, b0 + b1 made
// digit-wise (digits < 2^29, values < 2p: the SOS product's column sums stay below 2^62 and its output below 2p, since
// (2p)^2 < p 2^392): 4 unpacks instead of 6 and no Fp additions for the sums.  DG_FP2_DIG=1 (the one-wave pipeline
// kernels, where the digit arrays fit the register file) makes it fp2_mul's form; tests/test_host_arith.py checks it
// against fp2_mul on the host.
template <bool kSos = true>
DGI Fp fp28_product_packed(const uint32_t (&x)[14], const uint32_t (&y)[14]) {
  uint32_t d[14];
  if (kSos)
    fp28_sos_mul_d(x, y, d);
  else
    fp28_mont_mul_d(x, y, d);
  Fp r;
  fp28_pack(d, r.l);
  return fp_reduce_once(r);
}
#if defined(__HIP_DEVICE_COMPILE__)
#define DG_PIN_D14(d)                                                                                                 \
  asm volatile("" : "+v"((d)[0]), "+v"((d)[1]), "+v"((d)[2]), "+v"((d)[3]), "+v"((d)[4]), "+v"((d)[5]), "+v"((d)[6]), \
               "+v"((d)[7]), "+v"((d)[8]), "+v"((d)[9]), "+v"((d)[10]), "+v"((d)[11]), "+v"((d)[12]), "+v"((d)[13]))
#define DG_PIN_T12(f)                                                                                                 \
  asm volatile("" : "+v"((f).l[0]), "+v"((f).l[1]), "+v"((f).l[2]), "+v"((f).l[3]), "+v"((f).l[4]), "+v"((f).l[5]), \
               "+v"((f).l[6]), "+v"((f).l[7]), "+v"((f).l[8]), "+v"((f).l[9]), "+v"((f).l[10]), "+v"((f).l[11]))
#else
#define DG_PIN_D14(d) ((void)0)
#define DG_PIN_T12(f) ((void)0)
#endif
// (the three products serialised: each one's operands are pinned after the previous one's result)
template <bool kSos = true>
DGI Fp2 fp2_mul_dig(const Fp2& a, const Fp2& b) {
  uint32_t x0[14], x1[14], y0[14], y1[14], xs[14], ys[14];
  fp28_unpack(a.c0.l, x0);
  fp28_unpack(a.c1.l, x1);
  fp28_unpack(b.c0.l, y0);
  fp28_unpack(b.c1.l, y1);
#pragma unroll
  for (int i = 0; i < 14; ++i) {
    xs[i] = x0[i] + x1[i];
    ys[i] = y0[i] + y1[i];
  }
  Fp t0 = fp28_product_packed<kSos>(x0, y0);
  DG_PIN_T12(t0);
  DG_PIN_D14(x1);
  DG_PIN_D14(y1);
  Fp t1 = fp28_product_packed<kSos>(x1, y1);
  DG_PIN_T12(t1);
  DG_PIN_D14(xs);
  DG_PIN_D14(ys);
  const Fp t2 = fp28_product_packed<kSos>(xs, ys);
  return Fp2{fp_sub(t0, t1), fp_sub(fp_sub(t2, t0), t1)};
}
// fp2_mul_dig with two Montgomery reductions instead of three (the Karatsuba columns combined before reducing, as
// fpd.h fd2_mul): c0 = a0 b0 - a1 b1 from signed columns lies in (-p^2 / R, p^2 / R + p) for inputs below p, so p is
// added where the reduced top digit is negative and one conditional subtraction follows; c1 = a0 b1 + a1 b0 from the
// non-negative columns T2 - T0 - T1, below 2 p^2 / R + p.  The same values as fp2_mul (hostcheck.cpp)
DGI Fp2 fp2_mul_dig2(const Fp2& a, const Fp2& b) {
  uint32_t x0[14], x1[14], y0[14], y1[14];
  fp28_unpack(a.c0.l, x0);
  fp28_unpack(a.c1.l, x1);
  fp28_unpack(b.c0.l, y0);
  fp28_unpack(b.c1.l, y1);
  uint64_t d[27], s[27];
#pragma unroll
  for (int k = 0; k < 27; ++k) d[k] = s[k] = 0;
  fp28_cols(x0, y0, d);
  DG_PIN_D14(x1);
  DG_PIN_D14(y1);
  fp28_cols(x1, y1, s);
#pragma unroll
  for (int k = 0; k < 27; ++k) {
    const uint64_t t0 = d[k], t1 = s[k];
    d[k] = t0 - t1;
    s[k] = 0 - (t0 + t1);
  }
  uint32_t r[14];
  fp28_sos_reduce_signed(d, r);
  const uint32_t neg = (uint32_t)((int32_t)r[13] >> 31);
#pragma unroll
  for (int i = 0; i < 14; ++i) r[i] += P28[i] & neg;
#pragma unroll
  for (int i = 0; i < 13; ++i) {
    r[i + 1] += r[i] >> 28;
    r[i] &= FP28_MASK;
  }
  Fp c0;
  fp28_pack(r, c0.l);
  c0 = fp_reduce_once(c0);
  DG_PIN_T12(c0);
  uint32_t xs[14], ys[14];
#pragma unroll
  for (int i = 0; i < 14; ++i) {
    xs[i] = x0[i] + x1[i];
    ys[i] = y0[i] + y1[i];
  }
  fp28_cols(xs, ys, s);
  fp28_sos_reduce(s, r);
  Fp c1;
  fp28_pack(r, c1.l);
  return Fp2{c0, fp_reduce_once(c1)};
}
// a^2 = ((a0 + a1)(a0 - a1), 2 a0 a1): a0, a1 unpacked once, a0 + a1 digit-wise, a0 - a1 (mod p) unpacked
template <bool kSos = true>
DGI Fp2 fp2_sqr_dig(const Fp2& a) {
  uint32_t x0[14], x1[14], xs[14], xd[14];
  fp28_unpack(a.c0.l, x0);
  fp28_unpack(a.c1.l, x1);
  fp28_unpack(fp_sub(a.c0, a.c1).l, xd);
#pragma unroll
  for (int i = 0; i < 14; ++i) xs[i] = x0[i] + x1[i];
  Fp m = fp28_product_packed<kSos>(x0, x1);
  DG_PIN_T12(m);
  DG_PIN_D14(xs);
  DG_PIN_D14(xd);
  const Fp c0 = fp28_product_packed<kSos>(xs, xd);
  return Fp2{c0, fp_dbl(m)};
}
#ifndef DG_FP2_DIG
#define DG_FP2_DIG 0
#endif
DGH Fp2 fp2_mul(const Fp2& a, const Fp2& b) {
#if DG_FP2_DIG && DG_FP_CALL == 3 && defined(__HIP_DEVICE_COMPILE__)
  Fp2 x = a, y = b;
  DG_PIN_FP12(x.c0);
  DG_PIN_FP12(x.c1);
  DG_PIN_FP12(y.c0);
  DG_PIN_FP12(y.c1);
#if DG_FP2_DIG == 2
  Fp2 r = fp2_mul_dig2(x, y);  // two reductions
#else
  Fp2 r = fp2_mul_dig(x, y);
#endif
  DG_PIN_FP12(r.c0);
  DG_PIN_FP12(r.c1);
  return r;
#elif DG_FP2_PINNED
  Fp2 x = a, y = b;
  DG_PIN_FP12(x.c0);
  DG_PIN_FP12(x.c1);
  DG_PIN_FP12(y.c0);
  DG_PIN_FP12(y.c1);
  const Fp t0 = fp_mul_np(x.c0, y.c0);
  const Fp t1 = fp_mul_np(x.c1, y.c1);
  const Fp t2 = fp_mul_np(fp_add(x.c0, x.c1), fp_add(y.c0, y.c1));
  Fp2 r{fp_sub(t0, t1), fp_sub(fp_sub(t2, t0), t1)};
  DG_PIN_FP12(r.c0);
  DG_PIN_FP12(r.c1);
  return r;
#else
  Fp t0 = fp_mul(a.c0, b.c0);
  Fp t1 = fp_mul(a.c1, b.c1);
  Fp t2 = fp_mul(fp_add(a.c0, a.c1), fp_add(b.c0, b.c1));
  return Fp2{fp_sub(t0, t1), fp_sub(fp_sub(t2, t0), t1)};
#endif
}
DGH Fp2 fp2_sqr(const Fp2& a) {
#if DG_FP2_DIG && DG_FP_CALL == 3 && defined(__HIP_DEVICE_COMPILE__)
  Fp2 x = a;
  DG_PIN_FP12(x.c0);
  DG_PIN_FP12(x.c1);
  Fp2 r = fp2_sqr_dig(x);
  DG_PIN_FP12(r.c0);
  DG_PIN_FP12(r.c1);
  return r;
#elif DG_FP2_PINNED
  Fp2 x = a;
  DG_PIN_FP12(x.c0);
  DG_PIN_FP12(x.c1);
  const Fp m = fp_mul_np(x.c0, x.c1);
  Fp2 r{fp_mul_np(fp_add(x.c0, x.c1), fp_sub(x.c0, x.c1)), fp_dbl(m)};
  DG_PIN_FP12(r.c0);
  DG_PIN_FP12(r.c1);
  return r;
#else
  Fp m = fp_mul(a.c0, a.c1);
  return Fp2{fp_mul(fp_add(a.c0, a.c1), fp_sub(a.c0, a.c1)), fp_dbl(m)};
#endif
}
#endif
// Fp2 products as one out-of-line call each, operands and result in VGPRs (48 / 24 scalar arguments, the
// three or two Fp products inlined in the callee).  A caller of the Fp-level calls must keep its whole live set
// in the ~108 callee-saved VGPRs across every one of them (or spill it to scratch); across one Fp2-level call
// the Karatsuba temporaries stay inside the callee, so a curve formula's live set fits (g2_madd_lds).
#if defined(__HIP_DEVICE_COMPILE__) && DG_FP_CALL == 1
__device__ __noinline__ Fp2 fp2_mul_r(DG_P12(a), DG_P12(b), DG_P12(c), DG_P12(d)) {
  const Fp x0{{DG_L12(a)}}, x1{{DG_L12(b)}}, y0{{DG_L12(c)}}, y1{{DG_L12(d)}};
  const Fp t0 = fp28_mul(x0, y0);
  const Fp t1 = fp28_mul(x1, y1);
  const Fp t2 = fp28_mul(fp_add(x0, x1), fp_add(y0, y1));
  return Fp2{fp_sub(t0, t1), fp_sub(fp_sub(t2, t0), t1)};
}
__device__ __noinline__ Fp2 fp2_sqr_r(DG_P12(a), DG_P12(b)) {
  const Fp x0{{DG_L12(a)}}, x1{{DG_L12(b)}};
  const Fp m = fp28_mul(x0, x1);
  return Fp2{fp28_mul(fp_add(x0, x1), fp_sub(x0, x1)), fp_dbl(m)};
}
DGI Fp2 fp2_mul_rc(const Fp2& a, const Fp2& b) { return fp2_mul_r(DG_A12(a.c0), DG_A12(a.c1), DG_A12(b.c0), DG_A12(b.c1)); }
DGI Fp2 fp2_sqr_rc(const Fp2& a) { return fp2_sqr_r(DG_A12(a.c0), DG_A12(a.c1)); }
#else
DGI Fp2 fp2_mul_rc(const Fp2& a, const Fp2& b) { return fp2_mul(a, b); }
DGI Fp2 fp2_sqr_rc(const Fp2& a) { return fp2_sqr(a); }
#endif
// Inlined and serialised: each Fp product completes before the next one's operands are formed (DG_PIN_FP: an
// empty asm that reads and writes every limb, and volatile asms keep their order), so at most one product's
// temporaries are live -- the scheduler otherwise interleaves the three independent Karatsuba products and a
// curve formula around them outgrows 256 VGPRs (k_msm_aff_add: 300 VGPRs unserialised).
#if defined(__HIP_DEVICE_COMPILE__)
#define DG_PIN_FP(f)                                                                                                  \
  asm volatile("" : "+v"((f).l[0]), "+v"((f).l[1]), "+v"((f).l[2]), "+v"((f).l[3]), "+v"((f).l[4]), "+v"((f).l[5]), \
               "+v"((f).l[6]), "+v"((f).l[7]), "+v"((f).l[8]), "+v"((f).l[9]), "+v"((f).l[10]), "+v"((f).l[11]))
#else
#define DG_PIN_FP(f) ((void)0)
#endif
// DG_SEQ_SOS=1: the serialised product in the separated-operand-scanning form (fp28_sos_mul_d, as DG_FP_CALL=3),
// whose dependency chains are a few instructions long, instead of fp28_mul's column scan
#ifndef DG_SEQ_SOS
#define DG_SEQ_SOS 0
#endif
DGI Fp fp_mul_seq(Fp a, Fp b) {
  DG_PIN_FP(a);
  DG_PIN_FP(b);
#if DG_SEQ_SOS && defined(__HIP_DEVICE_COMPILE__)
  uint32_t x[14], y[14], d[14];
  fp28_unpack(a.l, x);
  fp28_unpack(b.l, y);
  fp28_sos_mul_d(x, y, d);
  Fp r;
  fp28_pack(d, r.l);
  r = fp_reduce_once(r);
#else
  Fp r = fp_mul_inl(a, b);
#endif
  DG_PIN_FP(r);
  return r;
}
// DG_SEQ_DIG=1: the serialised Fp2 forms in digit form (fp2_mul_dig / fp2_sqr_dig with the column-scan product; 2: with
// the SOS product)
#ifndef DG_SEQ_DIG
#define DG_SEQ_DIG 0
#endif
DGI Fp2 fp2_mul_seq(const Fp2& a, const Fp2& b) {
#if DG_SEQ_DIG && defined(__HIP_DEVICE_COMPILE__)
  {
    Fp2 x = a, y = b;
    DG_PIN_FP(x.c0);
    DG_PIN_FP(x.c1);
    DG_PIN_FP(y.c0);
    DG_PIN_FP(y.c1);
    Fp2 r = fp2_mul_dig<DG_SEQ_DIG == 2>(x, y);
    DG_PIN_FP(r.c0);
    DG_PIN_FP(r.c1);
    return r;
  }
#endif
  const Fp t0 = fp_mul_seq(a.c0, b.c0);
  const Fp t1 = fp_mul_seq(a.c1, b.c1);
  const Fp t2 = fp_mul_seq(fp_add(a.c0, a.c1), fp_add(b.c0, b.c1));
  return Fp2{fp_sub(t0, t1), fp_sub(fp_sub(t2, t0), t1)};
}
DGI Fp2 fp2_sqr_seq(const Fp2& a) {
#if DG_SEQ_DIG && defined(__HIP_DEVICE_COMPILE__)
  {
    Fp2 x = a;
    DG_PIN_FP(x.c0);
    DG_PIN_FP(x.c1);
    Fp2 r = fp2_sqr_dig<DG_SEQ_DIG == 2>(x);
    DG_PIN_FP(r.c0);
    DG_PIN_FP(r.c1);
    return r;
  }
#endif
  const Fp m = fp_mul_seq(a.c0, a.c1);
  return Fp2{fp_mul_seq(fp_add(a.c0, a.c1), fp_sub(a.c0, a.c1)), fp_dbl(m)};
}
// and inlined (the products' code at every call site)
DGI Fp2 fp2_mul_in(const Fp2& a, const Fp2& b) {
  const Fp t0 = fp_mul_inl(a.c0, b.c0);
  const Fp t1 = fp_mul_inl(a.c1, b.c1);
  const Fp t2 = fp_mul_inl(fp_add(a.c0, a.c1), fp_add(b.c0, b.c1));
  return Fp2{fp_sub(t0, t1), fp_sub(fp_sub(t2, t0), t1)};
}
DGI Fp2 fp2_sqr_in(const Fp2& a) {
  const Fp m = fp_mul_inl(a.c0, a.c1);
  return Fp2{fp_mul_inl(fp_add(a.c0, a.c1), fp_sub(a.c0, a.c1)), fp_dbl(m)};
}
DGI Fp2 fp2_mul_fp(const Fp2& a, const Fp& b) { return Fp2{fp_mul(a.c0, b), fp_mul(a.c1, b)}; }
DGI Fp2 fp2_mul_xi(const Fp2& a) { return Fp2{fp_sub(a.c0, a.c1), fp_add(a.c0, a.c1)}; }  // (1+u) a
DGI Fp fp2_norm(const Fp2& a) { return fp_add(fp_sqr(a.c0), fp_sqr(a.c1)); }
DGI Fp2 fp2_inv(const Fp2& a) {
  Fp n = fp_inv(fp2_norm(a));
  return Fp2{fp_mul(a.c0, n), fp_neg(fp_mul(a.c1, n))};
}
// RFC 9380 §4.1 sgn0 for m = 2
DGI uint32_t fp2_sgn0(const Fp2& a) {
  Fp x0 = fp_from_mont(a.c0);
  Fp x1 = fp_from_mont(a.c1);
  uint32_t sign0 = x0.l[0] & 1u;
  uint32_t zero0 = fp_is_zero(x0) ? 1u : 0u;
  uint32_t sign1 = x1.l[0] & 1u;
  return sign0 | (zero0 & sign1);
}
// ZCash sort flag for Fp2: c1 decides unless zero
DGI bool fp2_lex_largest(const Fp2& a) {
  Fp x1 = fp_from_mont(a.c1);
  if (!fp_is_zero(x1)) return fp_plain_gt_half(x1);
  return fp_plain_gt_half(fp_from_mont(a.c0));
}

// Square root in Fp2 with two Fp exponentiations ("complex method"):
//   s = sqrt(a0^2 + a1^2), c = (a0 + s)/2, t = c^((p-3)/4)
//   c square:      x = c t + (a1 t / 2) u
//   c non-square:  x = (a1 t / 2) - c t u           (since c t^2 = -1)
// `norm_sqrt` may be supplied by the caller (SSWU gx2 shortcut); result verified by squaring.
DGI bool fp2_sqrt_with_norm_root(Fp2& r, const Fp2& a, const Fp& s) {
  Fp half = fp_const(FP_TWO_INV);
  Fp x0, x1;
  if (fp_is_zero(a.c1)) {
    // a in Fp: sqrt(a0) or sqrt(-a0) * u
    Fp y;
    bool sq = fp_sqrt(y, a.c0);
    if (sq) {
      x0 = y;
      x1 = fp_zero();
    } else {
      fp_sqrt(y, fp_neg(a.c0));
      x0 = fp_zero();
      x1 = y;
    }
  } else {
    Fp c = fp_mul(fp_add(a.c0, s), half);
    Fp t = fp_pow_pm3d4(c);
    Fp ct = fp_mul(c, t);
    Fp at2 = fp_mul(fp_mul(a.c1, t), half);
    bool c_square = fp_eq(fp_mul(ct, t), fp_one());
    x0 = fp_sel(c_square, at2, ct);
    x1 = fp_sel(c_square, fp_neg(ct), at2);
  }
  r = Fp2{x0, x1};
  return fp2_eq(fp2_sqr(r), a);
}
DGI bool fp2_sqrt(Fp2& r, const Fp2& a) {
  Fp n = fp2_norm(a);
  Fp s;
  if (!fp_sqrt(s, n)) return false;
  return fp2_sqrt_with_norm_root(r, a, s);
}

// ------------------------------------------------------------------------------------------- Fp6
DGI Fp6 fp6_zero() { return Fp6{fp2_zero(), fp2_zero(), fp2_zero()}; }
DGI Fp6 fp6_add(const Fp6& a, const Fp6& b) { return Fp6{fp2_add(a.c0, b.c0), fp2_add(a.c1, b.c1), fp2_add(a.c2, b.c2)}; }
DGI Fp6 fp6_sub(const Fp6& a, const Fp6& b) { return Fp6{fp2_sub(a.c0, b.c0), fp2_sub(a.c1, b.c1), fp2_sub(a.c2, b.c2)}; }
DGI Fp6 fp6_neg(const Fp6& a) { return Fp6{fp2_neg(a.c0), fp2_neg(a.c1), fp2_neg(a.c2)}; }
DGI Fp6 fp6_mul_v(const Fp6& a) { return Fp6{fp2_mul_xi(a.c2), a.c0, a.c1}; }
DGH Fp6 fp6_mul(const Fp6& a, const Fp6& b) {
  Fp2 v0 = fp2_mul(a.c0, b.c0);
  Fp2 v1 = fp2_mul(a.c1, b.c1);
  Fp2 v2 = fp2_mul(a.c2, b.c2);
  Fp2 c0 = fp2_add(fp2_mul_xi(fp2_sub(fp2_sub(fp2_mul(fp2_add(a.c1, a.c2), fp2_add(b.c1, b.c2)), v1), v2)), v0);
  Fp2 c1 = fp2_add(fp2_sub(fp2_sub(fp2_mul(fp2_add(a.c0, a.c1), fp2_add(b.c0, b.c1)), v0), v1), fp2_mul_xi(v2));
  Fp2 c2 = fp2_add(fp2_sub(fp2_sub(fp2_mul(fp2_add(a.c0, a.c2), fp2_add(b.c0, b.c2)), v0), v2), v1);
  return Fp6{c0, c1, c2};
}
DGH Fp6 fp6_sqr(const Fp6& a) {
  // CH-SQR2
  Fp2 s0 = fp2_sqr(a.c0);
  Fp2 ab = fp2_mul(a.c0, a.c1);
  Fp2 s1 = fp2_dbl(ab);
  Fp2 s2 = fp2_sqr(fp2_add(fp2_sub(a.c0, a.c1), a.c2));
  Fp2 bc = fp2_mul(a.c1, a.c2);
  Fp2 s3 = fp2_dbl(bc);
  Fp2 s4 = fp2_sqr(a.c2);
  Fp2 c0 = fp2_add(fp2_mul_xi(s3), s0);
  Fp2 c1 = fp2_add(fp2_mul_xi(s4), s1);
  Fp2 c2 = fp2_sub(fp2_sub(fp2_add(fp2_add(s1, s2), s3), s0), s4);
  return Fp6{c0, c1, c2};
}
DG12 Fp6 fp6_inv(const Fp6& a) {
  Fp2 c0 = fp2_sub(fp2_sqr(a.c0), fp2_mul_xi(fp2_mul(a.c1, a.c2)));
  Fp2 c1 = fp2_sub(fp2_mul_xi(fp2_sqr(a.c2)), fp2_mul(a.c0, a.c1));
  Fp2 c2 = fp2_sub(fp2_sqr(a.c1), fp2_mul(a.c0, a.c2));
  Fp2 t = fp2_add(fp2_mul_xi(fp2_add(fp2_mul(a.c2, c1), fp2_mul(a.c1, c2))), fp2_mul(a.c0, c0));
  t = fp2_inv(t);
  return Fp6{fp2_mul(c0, t), fp2_mul(c1, t), fp2_mul(c2, t)};
}
// (a0 + a1 v + a2 v^2) * (b0 + b1 v)
DGH Fp6 fp6_mul_01(const Fp6& a, const Fp2& b0, const Fp2& b1) {
  Fp2 v0 = fp2_mul(a.c0, b0);
  Fp2 v1 = fp2_mul(a.c1, b1);
  Fp2 c0 = fp2_add(fp2_mul_xi(fp2_mul(a.c2, b1)), v0);
  Fp2 c1 = fp2_sub(fp2_sub(fp2_mul(fp2_add(a.c0, a.c1), fp2_add(b0, b1)), v0), v1);
  Fp2 c2 = fp2_add(fp2_mul(a.c2, b0), v1);
  return Fp6{c0, c1, c2};
}
// (a0 + a1 v + a2 v^2) * (b1 v)
DGI Fp6 fp6_mul_1(const Fp6& a, const Fp2& b1) {
  return Fp6{fp2_mul_xi(fp2_mul(a.c2, b1)), fp2_mul(a.c0, b1), fp2_mul(a.c1, b1)};
}

// ------------------------------------------------------------------------------------------- Fp12
DGI Fp12 fp12_one() { return Fp12{Fp6{fp2_one(), fp2_zero(), fp2_zero()}, fp6_zero()}; }
// DG_ML_INLINE: 0 keeps the Miller loop's sparse line product out of line; 1 (default) inlines it into the loop body
// of miller_loop (pairing.h); 2 also the line evaluations.  DG_ML_SQR_INLINE=1 inlines fp12_sqr as well.  Until
// round 3 fp12_sqr tested DG_ML_INLINE before the default was defined, so every shipped and measured build kept the
// squaring out of line; defining it inline grows the per-item kernels' private segment 11.4 -> 15.0 KB, so the
// default stays what was measured (0).
#ifndef DG_ML_INLINE
#define DG_ML_INLINE 1
#endif
#ifndef DG_ML_SQR_INLINE
#define DG_ML_SQR_INLINE 0
#endif
DGI bool fp12_is_one(const Fp12& a) {
  return fp2_eq(a.c0.c0, fp2_one()) && fp2_is_zero(a.c0.c1) && fp2_is_zero(a.c0.c2) && fp2_is_zero(a.c1.c0) &&
         fp2_is_zero(a.c1.c1) && fp2_is_zero(a.c1.c2);
}
DGI Fp12 fp12_conj(const Fp12& a) { return Fp12{a.c0, fp6_neg(a.c1)}; }
DG12 Fp12 fp12_mul(const Fp12& a, const Fp12& b) {
  Fp6 t0 = fp6_mul(a.c0, b.c0);
  Fp6 t1 = fp6_mul(a.c1, b.c1);
  Fp6 c1 = fp6_sub(fp6_sub(fp6_mul(fp6_add(a.c0, a.c1), fp6_add(b.c0, b.c1)), t0), t1);
  return Fp12{fp6_add(t0, fp6_mul_v(t1)), c1};
}
#if DG_ML_SQR_INLINE
DGI
#else
DG12
#endif
Fp12 fp12_sqr(const Fp12& a) {
  // complex squaring: (a0 + a1 w)^2 = (a0^2 + v a1^2) + 2 a0 a1 w
  Fp6 ab = fp6_mul(a.c0, a.c1);
  Fp6 s = fp6_mul(fp6_add(a.c0, a.c1), fp6_add(a.c0, fp6_mul_v(a.c1)));
  Fp6 c0 = fp6_sub(fp6_sub(s, ab), fp6_mul_v(ab));
  return Fp12{c0, fp6_add(ab, ab)};
}
DG12 Fp12 fp12_inv(const Fp12& a) {
  Fp6 t = fp6_sub(fp6_mul(a.c0, a.c0), fp6_mul_v(fp6_mul(a.c1, a.c1)));
  t = fp6_inv(t);
  return Fp12{fp6_mul(a.c0, t), fp6_neg(fp6_mul(a.c1, t))};
}
// Squaring in the cyclotomic subgroup (elements after the easy part of the final exponentiation), Granger-Scott:
// Fp12 seen as three Fp4 = Fp2[s]/(s^2 - xi) pieces (c0.c0, c1.c1), (c1.c0, c0.c2), (c0.c1, c1.c2); 9 Fp2
// squarings (18 Fp products) instead of the 36 of fp12_sqr.
// DG_CYC_SQR: the Fp2 squarings of fp4_sqr as Fp-level calls (0), inlined and serialised (1), inlined (2)
#ifndef DG_CYC_SQR
#define DG_CYC_SQR 2
#endif
#if DG_CYC_SQR == 1
#define DG_FP4_SQR2 fp2_sqr_seq
#elif DG_CYC_SQR == 2
#define DG_FP4_SQR2 fp2_sqr_in
#else
#define DG_FP4_SQR2 fp2_sqr
#endif
DGI void fp4_sqr(const Fp2& a, const Fp2& b, Fp2& c0, Fp2& c1) {
  Fp2 t0 = DG_FP4_SQR2(a), t1 = DG_FP4_SQR2(b);
  c0 = fp2_add(fp2_mul_xi(t1), t0);
  c1 = fp2_sub(fp2_sub(DG_FP4_SQR2(fp2_add(a, b)), t0), t1);
}
// DG_CYC_INLINE=1: inlined into its only caller, the loop of cyc_exp_z (the accumulator then stays in registers
// across the 63 squarings instead of crossing the call through the stack)
#ifndef DG_CYC_INLINE
#define DG_CYC_INLINE 1
#endif
#if DG_CYC_INLINE
DGI
#else
DG12
#endif
Fp12 fp12_cyc_sqr(const Fp12& f) {
  Fp2 z0 = f.c0.c0, z4 = f.c0.c1, z3 = f.c0.c2, z2 = f.c1.c0, z1 = f.c1.c1, z5 = f.c1.c2;
  Fp2 t0, t1, t2, t3;
  fp4_sqr(z0, z1, t0, t1);
  z0 = fp2_add(fp2_dbl(fp2_sub(t0, z0)), t0);  // 3 t0 - 2 z0
  z1 = fp2_add(fp2_dbl(fp2_add(t1, z1)), t1);  // 3 t1 + 2 z1
  fp4_sqr(z2, z3, t0, t1);
  fp4_sqr(z4, z5, t2, t3);
  z4 = fp2_add(fp2_dbl(fp2_sub(t0, z4)), t0);
  z5 = fp2_add(fp2_dbl(fp2_add(t1, z5)), t1);
  t0 = fp2_mul_xi(t3);
  z2 = fp2_add(fp2_dbl(fp2_add(t0, z2)), t0);
  z3 = fp2_add(fp2_dbl(fp2_sub(t2, z3)), t2);
  return Fp12{Fp6{z0, z4, z3}, Fp6{z2, z1, z5}};
}

// multiply by the sparse line l = c0 + c1 v + c4 v w (M-type twist; slots 0, 1, 4)
#if DG_ML_INLINE
DGI
#else
DG12
#endif
Fp12 fp12_mul_014(const Fp12& f, const Fp2& c0, const Fp2& c1, const Fp2& c4) {
  Fp6 aa = fp6_mul_01(f.c0, c0, c1);
  Fp6 bb = fp6_mul_1(f.c1, c4);
  Fp6 s = fp6_mul_01(fp6_add(f.c0, f.c1), c0, fp2_add(c1, c4));
  Fp6 n1 = fp6_sub(fp6_sub(s, aa), bb);
  Fp6 n0 = fp6_add(fp6_mul_v(bb), aa);
  return Fp12{n0, n1};
}
DG12 Fp12 fp12_frob(const Fp12& a) {
  Fp2 g1 = fp2_const(FROB_G1), g2 = fp2_const(FROB_G2), d = fp2_const(FROB_D);
  Fp6 b0{fp2_conj(a.c0.c0), fp2_mul(fp2_conj(a.c0.c1), g1), fp2_mul(fp2_conj(a.c0.c2), g2)};
  Fp2 dg1 = fp2_mul(d, g1), dg2 = fp2_mul(d, g2);
  Fp6 b1{fp2_mul(fp2_conj(a.c1.c0), d), fp2_mul(fp2_conj(a.c1.c1), dg1), fp2_mul(fp2_conj(a.c1.c2), dg2)};
  return Fp12{b0, b1};
}

}  // namespace dg
