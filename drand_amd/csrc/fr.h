// Scalar field Fr (r = 0x73eda753...00000001, 255 bits) for the Lagrange coefficients of Recover
// (A6/A12: kyber share.RecoverCommit interpolates at x = 0 over x_i = I + 1).
// 8 x 32-bit limbs, Montgomery form (R = 2^256).  Only a few hundred Fr multiplications run per
// recovered signature, so this is plain CIOS in C (no inline asm); the G2 scalar multiplications it
// feeds dominate by ~30x.
#pragma once
#include "field.h"

namespace dg {

struct Fr {
  uint32_t l[8];
};

DGI Fr fr_const(const uint32_t (&c)[8]) {
  Fr r;
#pragma unroll
  for (int i = 0; i < 8; ++i) r.l[i] = c[i];
  return r;
}
DGI Fr fr_sel(bool c, const Fr& a, const Fr& b) {
  Fr r;
#pragma unroll
  for (int i = 0; i < 8; ++i) r.l[i] = c ? b.l[i] : a.l[i];
  return r;
}
DGI Fr fr_reduce_once(const Fr& a) {
  Fr d;
  uint32_t br = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) d.l[i] = subb32(a.l[i], R_LIMBS[i], br, &br);
  return fr_sel(br == 0, a, d);
}
DGI Fr fr_sub(const Fr& a, const Fr& b) {
  Fr d;
  uint32_t br = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) d.l[i] = subb32(a.l[i], b.l[i], br, &br);
  uint32_t mask = 0u - br, c = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) d.l[i] = addc32(d.l[i], R_LIMBS[i] & mask, c, &c);
  return d;
}
DGI Fr fr_mul_in(const Fr& a, const Fr& b) {
  uint32_t t[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) t[j] = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    uint64_t p = (uint64_t)a.l[0] * b.l[i] + t[0];
    uint32_t A = (uint32_t)(p >> 32);
    uint32_t t0 = (uint32_t)p;
    uint32_t m = t0 * R_INV32;
    uint64_t q = (uint64_t)m * R_LIMBS[0] + t0;
    uint32_t C = (uint32_t)(q >> 32);
#pragma unroll
    for (int j = 1; j < 8; ++j) {
      p = (uint64_t)a.l[j] * b.l[i] + t[j] + A;
      A = (uint32_t)(p >> 32);
      q = (uint64_t)m * R_LIMBS[j] + (uint32_t)p + C;
      C = (uint32_t)(q >> 32);
      t[j - 1] = (uint32_t)q;
    }
    t[7] = C + A;
  }
  Fr r;
#pragma unroll
  for (int j = 0; j < 8; ++j) r.l[j] = t[j];
  return fr_reduce_once(r);
}
DGN Fr fr_mul(const Fr& a, const Fr& b) { return fr_mul_in(a, b); }
// small integer (< r) -> Montgomery
DGI Fr fr_from_u32(uint32_t v) {
  Fr a;
#pragma unroll
  for (int i = 0; i < 8; ++i) a.l[i] = 0;
  a.l[0] = v;
  return fr_mul(a, fr_const(FR_R2));
}
DGI Fr fr_to_plain(const Fr& a) {
  Fr one;
#pragma unroll
  for (int i = 0; i < 8; ++i) one.l[i] = 0;
  one.l[0] = 1;
  return fr_mul(a, one);
}
// a^(r-2) by the width-3 window schedule of tools/gen_constants.py (as fp_pow_sched); inline products, so a
// caller's frame holds no by-reference operands (an out-of-line fr_mul takes its operands through the stack)
DGI Fr fr_inv_in(const Fr& x) {
  Fr x2 = fr_mul_in(x, x);
  Fr t[4];
  t[0] = x;
#pragma unroll
  for (int i = 1; i < 4; ++i) t[i] = fr_mul_in(t[i - 1], x2);
  Fr acc = t[EXP_RM2_FIRST];
  for (int s = 0; s < EXP_RM2_NSTEPS; ++s) {
    int k = EXP_RM2_STEPS[s][0];
    int idx = EXP_RM2_STEPS[s][1];
    for (int j = 0; j < k; ++j) acc = fr_mul_in(acc, acc);
    if (idx >= 0) {
      Fr m = fr_sel(idx == 1, t[0], t[1]);
      m = fr_sel(idx == 2, m, t[2]);
      m = fr_sel(idx == 3, m, t[3]);
      acc = fr_mul_in(acc, m);
    }
  }
  return acc;
}
DGN Fr fr_inv(const Fr& x) { return fr_inv_in(x); }

// Lagrange coefficient at 0 of position j among the t interpolation points x_m = idx[m] + 1
// (kyber share.RecoverCommit / lagrangeBasis): lambda_j = prod_{m != j} x_m / (x_m - x_j).
// Returns the plain (non-Montgomery) scalar, little-endian limbs.  One lane per coefficient (k_rs_digits), so
// the products are inline and the factors enter in plain form: num and den each take t - 1 Montgomery products
// starting from R, so both carry the same R^(2-t) and it cancels in num / den (no per-factor conversion).
DGI Fr lagrange_at_zero(const uint32_t* idx, uint32_t t, uint32_t j) {
  Fr num = fr_const(FR_ONE), den = fr_const(FR_ONE), xj;
#pragma unroll
  for (int i = 0; i < 8; ++i) xj.l[i] = 0;
  xj.l[0] = idx[j] + 1;
  for (uint32_t m = 0; m < t; ++m) {
    if (m == j) continue;
    Fr xm = xj;
    xm.l[0] = idx[m] + 1;
    num = fr_mul_in(num, xm);
    den = fr_mul_in(den, fr_sub(xm, xj));
  }
  Fr one;
#pragma unroll
  for (int i = 0; i < 8; ++i) one.l[i] = 0;
  one.l[0] = 1;
  return fr_mul_in(fr_mul_in(num, fr_inv_in(den)), one);
}

}  // namespace dg
