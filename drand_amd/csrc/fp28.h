// 381-bit Montgomery multiplication / squaring with a radix-2^28 inner loop (host and device).
//
// Storage stays 12 x 32-bit limbs (field.h); the product works on 14 digits of 28 bits, so every
// 28 x 28-bit partial product is < 2^56 and a whole column -- at most 14 products of the operands,
// 14 of the Montgomery quotients and the carry -- sums below 2^61 in one 64-bit accumulator.  No carry
// propagation inside a column: on gfx950 each partial product is exactly one v_mad_u64_u32, against a
// v_mad_u64_u32 + v_addc_co_u32 pair in radix 2^32 (about 590 VALU instructions per multiplication
// instead of 755, +18% measured throughput: tools/microbench/r28.hip).
//
// Montgomery radix R = 2^392 (14 digits); every Montgomery-form constant is generated for it
// (tools/gen_constants.py).  Inputs < p give an output < 2p; the caller subtracts p once.
#pragma once
#include <stdint.h>

namespace dg {

constexpr uint32_t FP28_MASK = 0x0fffffffu;

// 12 x 32-bit limbs -> 14 x 28-bit digits
DGI void fp28_unpack(const uint32_t (&w)[12], uint32_t (&d)[14]) {
#pragma unroll
  for (int k = 0; k < 14; ++k) {
    const int bit = 28 * k, wi = bit >> 5, s = bit & 31;
    uint32_t lo = w[wi] >> s;
    if (s > 4 && wi + 1 < 12) lo |= w[wi + 1] << (32 - s);
    d[k] = lo & FP28_MASK;
  }
}
// 14 digits (the last one may hold up to 2^32 - 1 of carry) -> 12 x 32-bit limbs (value < 2^384)
DGI void fp28_pack(const uint32_t (&d)[14], uint32_t (&w)[12]) {
#pragma unroll
  for (int i = 0; i < 12; ++i) {
    const int bit = 32 * i, k = bit / 28, s = bit % 28;
    uint32_t v = d[k] >> s;
    v |= d[k + 1] << (28 - s);
    if (s > 24 && k + 2 < 14) v |= d[k + 2] << (56 - s);
    w[i] = v;
  }
}

// Column k of the Montgomery product scan: the quotient digits m_0..m_13 are produced in columns
// 0..13 (each zeroes the column's low 28 bits), columns 14..26 emit the result digits.
DGI void fp28_mont_tail(uint64_t& acc, int k, uint32_t (&m)[14], uint32_t (&r)[14]) {
#pragma unroll
  for (int i = 0; i < 14; ++i) {
    const int j = k - i;
    if (i < k && j >= 0 && j < 14) acc += (uint64_t)m[i] * P28[j];
  }
  if (k < 14) {
    m[k] = ((uint32_t)acc * P_INV28) & FP28_MASK;
    acc += (uint64_t)m[k] * P28[0];
  } else {
    r[k - 14] = (uint32_t)acc & FP28_MASK;
  }
  acc >>= 28;
}

// Digit form: 14 digits, digits 0..12 below 2^28, the top one below 2^20 (values < 2^384).  The
// products below take and return digit form, so an exponentiation chain stays in it between steps (no
// unpack / pack, no conditional subtraction: inputs < 2p give an output < 2p because 4p < R).

// r = x y / 2^392 mod p in digit form, r < 2p (x, y < 2p)
DGI void fp28_mont_mul_d(const uint32_t (&x)[14], const uint32_t (&y)[14], uint32_t (&r)[14]) {
  uint32_t m[14];
  uint64_t acc = 0;
#pragma unroll
  for (int k = 0; k < 27; ++k) {
#pragma unroll
    for (int i = 0; i < 14; ++i) {
      const int j = k - i;
      if (j >= 0 && j < 14) acc += (uint64_t)x[i] * y[j];
    }
    fp28_mont_tail(acc, k, m, r);
  }
  r[13] = (uint32_t)acc;
}

// r = x^2 / 2^392 mod p in digit form: the off-diagonal products once, doubled per column
DGI void fp28_mont_sqr_d(const uint32_t (&x)[14], uint32_t (&r)[14]) {
  uint32_t m[14];
  uint64_t acc = 0;
#pragma unroll
  for (int k = 0; k < 27; ++k) {
    uint64_t off = 0;
#pragma unroll
    for (int i = 0; i < 14; ++i) {
      const int j = k - i;
      if (j > i && j < 14) off += (uint64_t)x[i] * x[j];
    }
    acc += off << 1;
    if ((k & 1) == 0 && k / 2 < 14) acc += (uint64_t)x[k / 2] * x[k / 2];
    fp28_mont_tail(acc, k, m, r);
  }
  r[13] = (uint32_t)acc;
}

// Separated operand scanning (SOS) forms of the two products above, for the exponentiation kernel
// (phases.h): 27 lazy 64-bit column sums of the operand products, then 14 reduction rows of 14 independent
// multiply-adds each; every dependency chain is a few instructions long, so one wave keeps the SIMD's
// multiplier busy at the register count of a lean kernel (tools/microbench/expchain.hip: +4% over the
// single-accumulator scan at equal instruction count).  Same inputs / outputs / bounds as the _d forms.
DGI void fp28_sos_reduce(uint64_t (&t)[27], uint32_t (&r)[14]) {
#pragma unroll
  for (int i = 0; i < 14; ++i) {
    const uint32_t m = ((uint32_t)t[i] * P_INV28) & FP28_MASK;
#pragma unroll
    for (int j = 0; j < 14; ++j) t[i + j] += (uint64_t)m * P28[j];
    t[i + 1] += t[i] >> 28;
  }
#pragma unroll
  for (int k = 14; k < 26; ++k) {
    r[k - 14] = (uint32_t)t[k] & FP28_MASK;
    t[k + 1] += t[k] >> 28;
  }
  r[12] = (uint32_t)t[26] & FP28_MASK;
  r[13] = (uint32_t)(t[26] >> 28);
}
// fp28_sos_reduce for signed columns (two's complement in the 64-bit words): arithmetic carries, digits 0..12 below
// 2^28, the top one signed; the value is (T + m p) / 2^392 for the signed column value T (the two-reduction Fp2
// products: field.h fp2_mul_dig2, fpd.h fd2_mul)
DGI void fp28_sos_reduce_signed(uint64_t (&t)[27], uint32_t (&r)[14]) {
#pragma unroll
  for (int i = 0; i < 14; ++i) {
    const uint32_t m = ((uint32_t)t[i] * P_INV28) & FP28_MASK;
#pragma unroll
    for (int j = 0; j < 14; ++j) t[i + j] += (uint64_t)m * P28[j];
    t[i + 1] += (uint64_t)((int64_t)t[i] >> 28);
  }
#pragma unroll
  for (int k = 14; k < 26; ++k) {
    r[k - 14] = (uint32_t)t[k] & FP28_MASK;
    t[k + 1] += (uint64_t)((int64_t)t[k] >> 28);
  }
  r[12] = (uint32_t)t[26] & FP28_MASK;
  r[13] = (uint32_t)((int64_t)t[26] >> 28);
}
// t += x y as 27 column sums
DGI void fp28_cols(const uint32_t (&x)[14], const uint32_t (&y)[14], uint64_t (&t)[27]) {
#pragma unroll
  for (int i = 0; i < 14; ++i)
#pragma unroll
    for (int j = 0; j < 14; ++j) t[i + j] += (uint64_t)x[i] * y[j];
}
DGI void fp28_sos_mul_d(const uint32_t (&x)[14], const uint32_t (&y)[14], uint32_t (&r)[14]) {
  uint64_t t[27];
#pragma unroll
  for (int k = 0; k < 27; ++k) t[k] = 0;
#pragma unroll
  for (int i = 0; i < 14; ++i)
#pragma unroll
    for (int j = 0; j < 14; ++j) t[i + j] += (uint64_t)x[i] * y[j];
  fp28_sos_reduce(t, r);
}
DGI void fp28_sos_sqr_d(const uint32_t (&x)[14], uint32_t (&r)[14]) {
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
  fp28_sos_reduce(t, r);
}
// r = a b / 2^392 mod p, r < 2p (a, b < p)
DGI void fp28_mont_mul(const uint32_t (&a)[12], const uint32_t (&b)[12], uint32_t (&out)[12]) {
  uint32_t x[14], y[14], r[14];
  fp28_unpack(a, x);
  fp28_unpack(b, y);
  fp28_mont_mul_d(x, y, r);
  fp28_pack(r, out);
}

// r = a^2 / 2^392 mod p
DGI void fp28_mont_sqr(const uint32_t (&a)[12], uint32_t (&out)[12]) {
  uint32_t x[14], r[14];
  fp28_unpack(a, x);
  fp28_mont_sqr_d(x, r);
  fp28_pack(r, out);
}

}  // namespace dg
