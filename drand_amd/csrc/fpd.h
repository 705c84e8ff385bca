// Digit form through whole Fp12 operations (host and device): the Miller loops of the check pipeline (checks.h
// ck_miller_col) keep their accumulator and the line values as 14 digits of 28 bits -- the form the Montgomery
// products of fp28.h work in -- across every product, addition and subtraction of an Fp12 squaring or sparse line
// product, and convert only at the loop's edges.  field.h's 12-limb path unpacks the operands and packs the result of
// every product and reduces after every addition (~740 VALU instructions per product against the product's 392
// multiply-adds).
//
// Bounds (values in units of p; R = 2^392 ~ 2520 p):
//   - a product of inputs below X p and Y p is below (X Y / 2520 + 1) p: below 2 p for X, Y <= 40 (fp28 SOS form,
//     digits up to 2^29 -- one lazy addition -- keep every 64-bit column below 2^63);
//   - additions and subtractions leave digits normalised (below 2^28, the top one small); a - b adds the fat multiple
//     M p whose digits are all >= 2^28 - 1, so a + M p - b is digit-wise non-negative for any normalised b below M p;
//   - every Fp12 operation reduces its twelve outputs (fd_red: below 3 p) so the next one starts below 3 p.
// tests/native/hostcheck.cpp checks ck_miller_col against ck_miller with DG_FD_CHECK asserting the bounds.
#pragma once
#include "fp28.h"

namespace dg {

struct Fd {
  uint32_t d[14];
};
struct Fd2 {
  Fd c0, c1;
};
struct Fd6 {
  Fd2 c0, c1, c2;
};
struct Fd12 {
  Fd6 c0, c1;
};

namespace fdc {
constexpr uint32_t PD[14] = {0xfffaaab, 0xfefffff, 0x3ffffb9, 0xfffeb15, 0x6241eab, 0xa0f6b0f, 0xf6730d2,
                             0xf38512b, 0x4774b84, 0x4bacd76, 0xba7b643, 0xe69a4b1, 0x1ea397f, 0x1a011};
constexpr uint32_t PTOP_CEIL = 0x1a012;  // ceil(p / 2^364)
struct Fat {
  uint32_t k[14];
};
// M p with digits k_0 = c_0 + 2^28, k_i = c_i + 2^28 - 1 (0 < i < 13), k_13 = c_13 - 1 (the same value)
constexpr Fat fat(uint32_t M) {
  Fat r{};
  uint64_t carry = 0;
  uint32_t c[14] = {};
  for (int i = 0; i < 13; ++i) {
    const uint64_t v = (uint64_t)PD[i] * M + carry;
    c[i] = (uint32_t)(v & 0x0fffffffu);
    carry = v >> 28;
  }
  c[13] = (uint32_t)((uint64_t)PD[13] * M + carry);
  r.k[0] = c[0] + (1u << 28);
  for (int i = 1; i < 13; ++i) r.k[i] = c[i] + (1u << 28) - 1;
  r.k[13] = c[13] - 1;
  return r;
}
}  // namespace fdc

#if defined(DG_FD_CHECK) && !defined(__HIP_DEVICE_COMPILE__)
// host builds of the checks: value < 2^hi_bits p-ish bound via the top digit, digits below 2^lim
void fd_check_fail(const char* what);
#define DG_FD_ASSERT(c, what) \
  do {                        \
    if (!(c)) fd_check_fail(what); \
  } while (0)
#else
#define DG_FD_ASSERT(c, what) ((void)0)
#endif

DGI void fd_norm(Fd& a) {
#pragma unroll
  for (int i = 0; i < 13; ++i) {
    a.d[i + 1] += a.d[i] >> 28;
    a.d[i] &= FP28_MASK;
  }
}
DGI Fd fd_from(const Fp& a) {
  Fd r;
  fp28_unpack(a.l, r.d);
  return r;
}
DGI Fd fd_zero() {
  Fd r;
#pragma unroll
  for (int i = 0; i < 14; ++i) r.d[i] = 0;
  return r;
}
DGI Fd fd_add(const Fd& a, const Fd& b) {
  Fd r;
#pragma unroll
  for (int i = 0; i < 14; ++i) r.d[i] = a.d[i] + b.d[i];
  fd_norm(r);
  return r;
}
// a + b without carries: digits below 2^29, only as an operand of fd_mul / fd_sqr
DGI Fd fd_add_lazy(const Fd& a, const Fd& b) {
  Fd r;
#pragma unroll
  for (int i = 0; i < 14; ++i) r.d[i] = a.d[i] + b.d[i];
  return r;
}
// a - b + M p (b normalised and below M p)
template <uint32_t M>
DGI Fd fd_sub(const Fd& a, const Fd& b) {
  constexpr fdc::Fat K = fdc::fat(M);
  Fd r;
#pragma unroll
  for (int i = 0; i < 14; ++i) r.d[i] = a.d[i] + K.k[i] - b.d[i];
  DG_FD_ASSERT(b.d[13] < K.k[13], "fd_sub: subtrahend above M p");
  fd_norm(r);
  return r;
}
template <uint32_t M>
DGI Fd fd_neg(const Fd& a) {
  return fd_sub<M>(fd_zero(), a);
}
DGI Fd fd_dbl(const Fd& a) { return fd_add(a, a); }
// The products are serialised (operands and result pinned by empty asm statements, which keep their program order):
// without that the compiler interleaves a whole Fp6 product's operands and spills (401 VGPRs spilled in k_ck_miller).
DGI Fd fd_mul(const Fd& a, const Fd& b) {
  DG_FD_ASSERT(a.d[13] < (1u << 25) && b.d[13] < (1u << 25), "fd_mul: operand too large");
  Fd x = a, y = b, r;
  DG_PIN_D14(x.d);
  DG_PIN_D14(y.d);
  fp28_sos_mul_d(x.d, y.d, r.d);
  DG_PIN_D14(r.d);
  return r;
}
DGI Fd fd_sqr(const Fd& a) {
  DG_FD_ASSERT(a.d[13] < (1u << 25), "fd_sqr: operand too large");
  Fd x = a, r;
  DG_PIN_D14(x.d);
  fp28_sos_sqr_d(x.d, r.d);
  DG_PIN_D14(r.d);
  return r;
}
// a mod p up to a small multiple: a - q p, q = floor(top digit / ceil(p / 2^364)) <= a / p; below 3 p
DGI Fd fd_red(const Fd& a) {
  const uint32_t q = a.d[13] / fdc::PTOP_CEIL;
  Fd r;
  int64_t c = 0;
#pragma unroll
  for (int i = 0; i < 13; ++i) {
    const int64_t v = (int64_t)a.d[i] - (int64_t)q * fdc::PD[i] + c;
    r.d[i] = (uint32_t)v & FP28_MASK;
    c = v >> 28;
  }
  r.d[13] = (uint32_t)((int64_t)a.d[13] - (int64_t)q * fdc::PD[13] + c);
  DG_FD_ASSERT(r.d[13] <= 3u * fdc::PD[13] + 3u, "fd_red: result above 3 p");
  return r;
}
// back to 12 limbs, fully reduced
DGI Fp fd_to(const Fd& a) {
  const Fd r = fd_red(a);
  Fp o;
  fp28_pack(r.d, o.l);
  return fp_reduce_once(fp_reduce_once(o));
}

// ---- Fp2 = Fp[u] / (u^2 + 1)
DGI Fd2 fd2_from(const Fp2& a) { return Fd2{fd_from(a.c0), fd_from(a.c1)}; }
DGI Fp2 fd2_to(const Fd2& a) { return Fp2{fd_to(a.c0), fd_to(a.c1)}; }
DGI Fd2 fd2_add(const Fd2& a, const Fd2& b) { return Fd2{fd_add(a.c0, b.c0), fd_add(a.c1, b.c1)}; }
template <uint32_t M>
DGI Fd2 fd2_sub(const Fd2& a, const Fd2& b) {
  return Fd2{fd_sub<M>(a.c0, b.c0), fd_sub<M>(a.c1, b.c1)};
}
DGI Fd2 fd2_red(const Fd2& a) { return Fd2{fd_red(a.c0), fd_red(a.c1)}; }
// inputs below 40 p: c0 below 6 p, c1 below 10 p (three reductions: the form fd2_mul replaced, kept for the host check)
DGI Fd2 fd2_mul3(const Fd2& a, const Fd2& b) {
  const Fd t0 = fd_mul(a.c0, b.c0), t1 = fd_mul(a.c1, b.c1);
  const Fd t2 = fd_mul(fd_add_lazy(a.c0, a.c1), fd_add_lazy(b.c0, b.c1));
  Fd2 r{fd_sub<4>(t0, t1), fd_sub<8>(t2, fd_add(t0, t1))};
  DG_PIN_D14(r.c0.d);
  DG_PIN_D14(r.c1.d);
  return r;
}
// Fp2 product with two Montgomery reductions instead of three (~15% fewer instructions): the Karatsuba columns are
// combined before reducing.  c0 = a0 b0 - a1 b1 from signed columns: |a0 b0 - a1 b1| < 1600 p^2 for inputs below 40 p,
// so the reduced value lies in (-0.64 p, 1.64 p) (R ~ 2520 p), and 2 p added digit-wise (the top digit wrapping modulo
// 2^32 back to the true non-negative value) leaves it below 3.7 p.  c1 = (a0 + a1)(b0 + b1) - (a0 b0 + a1 b1): the
// columns of a0 b1 + a1 b0, non-negative; below 2.3 p.  Same bound contract as fd2_mul3 (tighter outputs).
DGI Fd2 fd2_mul(const Fd2& a, const Fd2& b) {
  DG_FD_ASSERT(a.c0.d[13] < (1u << 25) && a.c1.d[13] < (1u << 25) && b.c0.d[13] < (1u << 25) &&
                   b.c1.d[13] < (1u << 25),
               "fd2_mul: operand too large");
  Fd x0 = a.c0, x1 = a.c1, y0 = b.c0, y1 = b.c1;
  DG_PIN_D14(x0.d);
  DG_PIN_D14(y0.d);
  uint64_t d[27], s[27];
#pragma unroll
  for (int k = 0; k < 27; ++k) d[k] = s[k] = 0;
  fp28_cols(x0.d, y0.d, d);
  DG_PIN_D14(x1.d);
  DG_PIN_D14(y1.d);
  fp28_cols(x1.d, y1.d, s);
#pragma unroll
  for (int k = 0; k < 27; ++k) {
    const uint64_t t0 = d[k], t1 = s[k];
    d[k] = t0 - t1;
    s[k] = 0 - (t0 + t1);
  }
  Fd2 r;
  fp28_sos_reduce_signed(d, r.c0.d);
  constexpr fdc::Fat P2 = fdc::fat(2);  // 2 p with every digit >= 2^28 - 1 (digit-wise addition, then carries)
#pragma unroll
  for (int i = 0; i < 14; ++i) r.c0.d[i] += P2.k[i];
  fd_norm(r.c0);
  DG_PIN_D14(r.c0.d);
  const Fd xs = fd_add_lazy(x0, x1), ys = fd_add_lazy(y0, y1);
  fp28_cols(xs.d, ys.d, s);
  fp28_sos_reduce(s, r.c1.d);
  DG_PIN_D14(r.c1.d);
  DG_FD_ASSERT(r.c0.d[13] <= 4u * fdc::PD[13] && r.c1.d[13] <= 3u * fdc::PD[13], "fd2_mul: output above bound");
  return r;
}
// (a0 + a1)(a0 - a1), 2 a0 a1 (inputs below 20 p): c0 below 2 p, c1 below 4 p
DGI Fd2 fd2_sqr(const Fd2& a) {
  const Fd m = fd_mul(a.c0, a.c1);
  const Fd c0 = fd_mul(fd_add_lazy(a.c0, a.c1), fd_sub<32>(a.c0, a.c1));
  return Fd2{c0, fd_dbl(m)};
}
// (1 + u) a = (a0 - a1, a0 + a1), a1 below M p
template <uint32_t M>
DGI Fd2 fd2_mul_xi(const Fd2& a) {
  return Fd2{fd_sub<M>(a.c0, a.c1), fd_add(a.c0, a.c1)};
}
DGI Fd2 fd2_mul_fp(const Fd2& a, const Fd& b) { return Fd2{fd_mul(a.c0, b), fd_mul(a.c1, b)}; }

// ---- Fp6 = Fp2[v] / (v^3 - xi) (field.h fp6_mul / fp6_mul_01 / fp6_mul_1 formulas); inputs below 20 p
DGI Fd6 fd6_add(const Fd6& a, const Fd6& b) { return Fd6{fd2_add(a.c0, b.c0), fd2_add(a.c1, b.c1), fd2_add(a.c2, b.c2)}; }
template <uint32_t M>
DGI Fd6 fd6_sub(const Fd6& a, const Fd6& b) {
  return Fd6{fd2_sub<M>(a.c0, b.c0), fd2_sub<M>(a.c1, b.c1), fd2_sub<M>(a.c2, b.c2)};
}
template <uint32_t M>
DGI Fd6 fd6_mul_v(const Fd6& a) {
  return Fd6{fd2_mul_xi<M>(a.c2), a.c0, a.c1};
}
// outputs below ~70 p (each Fd2 product below 10 p)
// (each cross product consumed as soon as it is formed: a smaller live set)
DGI Fd6 fd6_mul(const Fd6& a, const Fd6& b) {
  const Fd2 v0 = fd2_mul(a.c0, b.c0), v1 = fd2_mul(a.c1, b.c1), v2 = fd2_mul(a.c2, b.c2);
  const Fd2 c0 = fd2_add(fd2_mul_xi<64>(fd2_sub<32>(fd2_mul(fd2_add(a.c1, a.c2), fd2_add(b.c1, b.c2)), fd2_add(v1, v2))), v0);
  const Fd2 c1 = fd2_add(fd2_sub<32>(fd2_mul(fd2_add(a.c0, a.c1), fd2_add(b.c0, b.c1)), fd2_add(v0, v1)), fd2_mul_xi<16>(v2));
  const Fd2 c2 = fd2_add(fd2_sub<32>(fd2_mul(fd2_add(a.c0, a.c2), fd2_add(b.c0, b.c2)), fd2_add(v0, v2)), v1);
  return Fd6{c0, c1, c2};
}
// (a0 + a1 v + a2 v^2)(b0 + b1 v)
DGI Fd6 fd6_mul_01(const Fd6& a, const Fd2& b0, const Fd2& b1) {
  const Fd2 v0 = fd2_mul(a.c0, b0), v1 = fd2_mul(a.c1, b1);
  const Fd2 c0 = fd2_add(fd2_mul_xi<16>(fd2_mul(a.c2, b1)), v0);
  const Fd2 c1 = fd2_sub<32>(fd2_mul(fd2_add(a.c0, a.c1), fd2_add(b0, b1)), fd2_add(v0, v1));
  const Fd2 c2 = fd2_add(fd2_mul(a.c2, b0), v1);
  return Fd6{c0, c1, c2};
}
// (a0 + a1 v + a2 v^2)(b1 v)
DGI Fd6 fd6_mul_1(const Fd6& a, const Fd2& b1) {
  return Fd6{fd2_mul_xi<16>(fd2_mul(a.c2, b1)), fd2_mul(a.c0, b1), fd2_mul(a.c1, b1)};
}
DGI Fd6 fd6_red(const Fd6& a) { return Fd6{fd2_red(a.c0), fd2_red(a.c1), fd2_red(a.c2)}; }
// materialise an intermediate (the formulas below are ordered so that operands die early)
DGI void fd6_pin(Fd6& a) {
  DG_PIN_D14(a.c0.c0.d);
  DG_PIN_D14(a.c0.c1.d);
  DG_PIN_D14(a.c1.c0.d);
  DG_PIN_D14(a.c1.c1.d);
  DG_PIN_D14(a.c2.c0.d);
  DG_PIN_D14(a.c2.c1.d);
}


// ---- Fp12 = Fp6[w] / (w^2 - v); every operation returns its outputs reduced (below 3 p)
DGI Fd12 fd12_from(const Fp12& a) {
  return Fd12{Fd6{fd2_from(a.c0.c0), fd2_from(a.c0.c1), fd2_from(a.c0.c2)},
              Fd6{fd2_from(a.c1.c0), fd2_from(a.c1.c1), fd2_from(a.c1.c2)}};
}
DGI Fp12 fd12_to(const Fd12& a) {
  return Fp12{Fp6{fd2_to(a.c0.c0), fd2_to(a.c0.c1), fd2_to(a.c0.c2)},
              Fp6{fd2_to(a.c1.c0), fd2_to(a.c1.c1), fd2_to(a.c1.c2)}};
}
// (a0 + a1 w)^2 = (s - ab - v ab) + 2 ab w, s = (a0 + a1)(a0 + v a1)  (field.h fp12_sqr)
DGI Fd12 fd12_sqr(const Fd12& a) {
  Fd6 ab = fd6_mul(a.c0, a.c1);
  fd6_pin(ab);
  Fd6 x = fd6_add(a.c0, a.c1), y = fd6_add(a.c0, fd6_mul_v<4>(a.c1));
  fd6_pin(x);
  fd6_pin(y);
  const Fd6 s = fd6_mul(x, y);
  const Fd6 c0 = fd6_sub<256>(fd6_sub<128>(s, ab), fd6_mul_v<128>(ab));
  return Fd12{fd6_red(c0), fd6_red(fd6_add(ab, ab))};
}
// f (c0 + c1 v + c4 v w)  (field.h fp12_mul_014)
// (aa from f.c0, then the sum -- f.c0 dead -- then bb from f.c1 -- f dead -- then s)
DGI Fd12 fd12_mul_014(const Fd12& f, const Fd2& c0, const Fd2& c1, const Fd2& c4) {
  Fd6 aa = fd6_mul_01(f.c0, c0, c1);
  fd6_pin(aa);
  Fd6 t = fd6_add(f.c0, f.c1);
  fd6_pin(t);
  Fd6 bb = fd6_mul_1(f.c1, c4);
  fd6_pin(bb);
  const Fd6 s = fd6_mul_01(t, c0, fd2_add(c1, c4));
  const Fd6 n1 = fd6_sub<128>(s, fd6_add(aa, bb));
  const Fd6 n0 = fd6_add(fd6_mul_v<64>(bb), aa);
  return Fd12{fd6_red(n0), fd6_red(n1)};
}
DGI Fd12 fd12_one() {
  const Fd one = fd_from(fp_one()), z = fd_zero();
  return Fd12{Fd6{Fd2{one, z}, Fd2{z, z}, Fd2{z, z}}, Fd6{Fd2{z, z}, Fd2{z, z}, Fd2{z, z}}};
}

// ---- an Fp12 accumulator outside the register file (checks.h k_ck_miller: one LDS column per lane, 576 B)
// Component i (0..11, the Fd12 order c0.c0.c0, c0.c0.c1, c0.c1.c0, ...) is 12 limbs of a value below 3 p (fd_red, not
// fully reduced: 3 p < 2^384) at w[(12 i + k) kStride]; lanes of a wave read consecutive words (kStride = the lanes).
// The loop's live set is then the operation's own temporaries: the 168 digit registers of the accumulator are what
// made the register form of this loop spill (213-430 VGPRs).
#define DG_FD_RELOAD() asm volatile("" ::: "memory")  // a later get() reads the column again (no live copy kept)
#if defined(__HIP__)
#define DG_MEMBER __host__ __device__ __forceinline__
#else
#define DG_MEMBER inline
#endif
template <uint32_t kStride>
struct Fd12Col {
  uint32_t* w;
  DG_MEMBER Fd get(int i) const {
    uint32_t l[12];
#pragma unroll
    for (int k = 0; k < 12; ++k) l[k] = w[(size_t)(12 * i + k) * kStride];
    return fd_from(Fp{{l[0], l[1], l[2], l[3], l[4], l[5], l[6], l[7], l[8], l[9], l[10], l[11]}});
  }
  DG_MEMBER void put(int i, const Fd& a) {
    const Fd r = fd_red(a);
    uint32_t l[12];
    fp28_pack(r.d, l);
#pragma unroll
    for (int k = 0; k < 12; ++k) w[(size_t)(12 * i + k) * kStride] = l[k];
  }
  DG_MEMBER Fd6 get6(int h) const {
    return Fd6{Fd2{get(6 * h), get(6 * h + 1)}, Fd2{get(6 * h + 2), get(6 * h + 3)}, Fd2{get(6 * h + 4), get(6 * h + 5)}};
  }
  DG_MEMBER void put6(int h, const Fd6& a) {
    put(6 * h, a.c0.c0);
    put(6 * h + 1, a.c0.c1);
    put(6 * h + 2, a.c1.c0);
    put(6 * h + 3, a.c1.c1);
    put(6 * h + 4, a.c2.c0);
    put(6 * h + 5, a.c2.c1);
  }
  DG_MEMBER void set_one() {
    const Fd one = fd_from(fp_one()), z = fd_zero();
    put(0, one);
#pragma unroll 1
    for (int i = 1; i < 12; ++i) put(i, z);
  }
  DG_MEMBER Fp12 to_fp12() const {
    Fp c[12];
#pragma unroll
    for (int i = 0; i < 12; ++i) c[i] = fd_to(get(i));
    return Fp12{Fp6{Fp2{c[0], c[1]}, Fp2{c[2], c[3]}, Fp2{c[4], c[5]}}, Fp6{Fp2{c[6], c[7]}, Fp2{c[8], c[9]}, Fp2{c[10], c[11]}}};
  }
};
// fd12_sqr on a column: the same formula and bounds; each half is loaded where it is used (twice, instead of a live
// copy beside the products) and the outputs stored as they are formed
template <class C>
DGI void fd12_sqr_col(C& f) {
  Fd6 ab;
  {
    const Fd6 a0 = f.get6(0), a1 = f.get6(1);
    ab = fd6_mul(a0, a1);
  }
  fd6_pin(ab);
  DG_FD_RELOAD();
  Fd6 x, y;
  {
    const Fd6 a0 = f.get6(0), a1 = f.get6(1);
    x = fd6_add(a0, a1);
    y = fd6_add(a0, fd6_mul_v<4>(a1));
  }
  fd6_pin(x);
  fd6_pin(y);
  f.put6(1, fd6_add(ab, ab));
  const Fd6 s = fd6_mul(x, y);
  f.put6(0, fd6_sub<256>(fd6_sub<128>(s, ab), fd6_mul_v<128>(ab)));
  DG_FD_RELOAD();
}
// fd12_mul_014 on a column (n0 = v bb + aa, n1 = s - (aa + bb), s = (f0 + f1)(c0 + (c1 + c4) v))
template <class C>
DGI void fd12_mul_014_col(C& f, const Fd2& c0, const Fd2& c1, const Fd2& c4) {
  Fd6 bb = fd6_mul_1(f.get6(1), c4);
  fd6_pin(bb);
  DG_FD_RELOAD();
  Fd6 aa = fd6_mul_01(f.get6(0), c0, c1);
  fd6_pin(aa);
  Fd6 u = fd6_add(aa, bb);
  fd6_pin(u);
  Fd6 n0 = fd6_add(fd6_mul_v<64>(bb), aa);
  fd6_pin(n0);
  DG_FD_RELOAD();
  Fd6 t = fd6_add(f.get6(0), f.get6(1));
  fd6_pin(t);
  f.put6(0, n0);
  const Fd6 s = fd6_mul_01(t, c0, fd2_add(c1, c4));
  f.put6(1, fd6_sub<128>(s, u));
  DG_FD_RELOAD();
}

}  // namespace dg
