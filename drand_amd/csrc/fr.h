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
// CIOS over the NB low limbs of b: a b 2^(-32 NB) mod r (NB = 8: the Montgomery product).  After each limb the
// partial result is < 2r (a < r, r < 2^255), so the top limb never carries out and one reduction ends it.
template <int NB>
DGI Fr fr_cios(const Fr& a, const uint32_t* b) {
  uint32_t t[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) t[j] = 0;
#pragma unroll
  for (int i = 0; i < NB; ++i) {
    uint64_t p = (uint64_t)a.l[0] * b[i] + t[0];
    uint32_t A = (uint32_t)(p >> 32);
    uint32_t t0 = (uint32_t)p;
    uint32_t m = t0 * R_INV32;
    uint64_t q = (uint64_t)m * R_LIMBS[0] + t0;
    uint32_t C = (uint32_t)(q >> 32);
#pragma unroll
    for (int j = 1; j < 8; ++j) {
      p = (uint64_t)a.l[j] * b[i] + t[j] + A;
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
DGI Fr fr_mul_in(const Fr& a, const Fr& b) { return fr_cios<8>(a, b.l); }
// a b 2^-64 for a plain 64-bit b: a quarter of a Montgomery product
DGI Fr fr_mul_u64(const Fr& a, uint64_t b) {
  const uint32_t bl[2] = {(uint32_t)b, (uint32_t)(b >> 32)};
  return fr_cios<2>(a, bl);
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
// The factors are small integers, multiplied in plain 64-bit chunks (x_m and |x_m - x_j| side by side, a chunk
// closed when either would pass 64 bits) and each pair of chunks entered by one fr_mul_u64: num and den take the
// same number of 2^-64 factors from the Montgomery one R, so they cancel in num / den -- at k = 256 about 19
// quarter-products per coefficient instead of 2 (t - 1) full ones.  den's sign is the parity of the x_m < x_j.
DGI uint32_t u64_bits(uint64_t v) { return v ? 64u - (uint32_t)__builtin_clzll(v) : 0u; }
DGI void lagrange_nd(const uint32_t* idx, uint32_t t, uint32_t j, Fr& num, Fr& den) {
  num = fr_const(FR_ONE);
  den = num;
  const uint64_t xj = (uint64_t)idx[j] + 1;
  uint64_t cn = 1, cd = 1;
  uint32_t neg = 0;
  for (uint32_t m = 0; m < t; ++m) {
    if (m == j) continue;
    const uint64_t xm = (uint64_t)idx[m] + 1;
    const uint64_t d = xm > xj ? xm - xj : xj - xm;
    neg ^= xm < xj ? 1u : 0u;
    if (u64_bits(cn) + u64_bits(xm) > 64 || u64_bits(cd) + u64_bits(d) > 64) {
      num = fr_mul_u64(num, cn);
      den = fr_mul_u64(den, cd);
      cn = xm;
      cd = d;
    } else {
      cn *= xm;
      cd *= d;
    }
  }
  num = fr_mul_u64(num, cn);
  den = fr_mul_u64(den, cd);
  if (neg) {
    Fr z;
#pragma unroll
    for (int i = 0; i < 8; ++i) z.l[i] = 0;
    den = fr_sub(z, den);
  }
}
// lambda_j from lagrange_nd's pair and 1 / den (both Montgomery): the plain scalar
DGI Fr lagrange_finish(const Fr& num, const Fr& dinv) {
  Fr one;
#pragma unroll
  for (int i = 0; i < 8; ++i) one.l[i] = 0;
  one.l[0] = 1;
  return fr_mul_in(fr_mul_in(num, dinv), one);
}
// Returns the plain (non-Montgomery) scalar, little-endian limbs.
DGI Fr lagrange_at_zero(const uint32_t* idx, uint32_t t, uint32_t j) {
  Fr num, den;
  lagrange_nd(idx, t, j, num, den);
  return lagrange_finish(num, fr_inv_in(den));
}

}  // namespace dg
