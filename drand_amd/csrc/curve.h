// G1 (over Fp) and G2 (over Fp2, the sextic M-twist E': y^2 = x^3 + 4(1+u)) group arithmetic.
// Jacobian coordinates (x = X/Z^2, y = Y/Z^3), Z = 0 is the point at infinity.
// ZCash compressed encodings (G1 48 B, G2 96 B with x = c1 || c0; flags 0x80 compressed,
// 0x40 infinity, 0x20 "y lexicographically largest") as produced by kyber's MarshalBinary for the
// suite chosen at key/curve.go:12 (keys on G1 key/curve.go:21, signatures on G2 key/curve.go:26).
#pragma once
#include "field.h"

namespace dg {

// ---- field-generic helpers so one template serves G1 and G2
DGI Fp f_add(const Fp& a, const Fp& b) { return fp_add(a, b); }
DGI Fp f_sub(const Fp& a, const Fp& b) { return fp_sub(a, b); }
DGI Fp f_mul(const Fp& a, const Fp& b) { return fp_mul(a, b); }
DGI Fp f_sqr(const Fp& a) { return fp_sqr(a); }
DGI Fp f_dbl(const Fp& a) { return fp_dbl(a); }
DGI Fp f_neg(const Fp& a) { return fp_neg(a); }
DGI bool f_is_zero(const Fp& a) { return fp_is_zero(a); }
DGI bool f_eq(const Fp& a, const Fp& b) { return fp_eq(a, b); }
DGI Fp f_sel(bool c, const Fp& a, const Fp& b) { return fp_sel(c, a, b); }
DGI Fp2 f_add(const Fp2& a, const Fp2& b) { return fp2_add(a, b); }
DGI Fp2 f_sub(const Fp2& a, const Fp2& b) { return fp2_sub(a, b); }
DGI Fp2 f_mul(const Fp2& a, const Fp2& b) { return fp2_mul(a, b); }
DGI Fp2 f_sqr(const Fp2& a) { return fp2_sqr(a); }
DGI Fp2 f_dbl(const Fp2& a) { return fp2_dbl(a); }
DGI Fp2 f_neg(const Fp2& a) { return fp2_neg(a); }
DGI bool f_is_zero(const Fp2& a) { return fp2_is_zero(a); }
DGI bool f_eq(const Fp2& a, const Fp2& b) { return fp2_eq(a, b); }
DGI Fp2 f_sel(bool c, const Fp2& a, const Fp2& b) { return fp2_sel(c, a, b); }

template <class F>
struct Jac {
  F x, y, z;
};
template <class F>
struct Aff {
  F x, y;
  bool inf;
};
typedef Jac<Fp> G1J;
typedef Jac<Fp2> G2J;
typedef Aff<Fp> G1A;
typedef Aff<Fp2> G2A;

DGI Fp f_zero_of(const Fp&) { return fp_zero(); }
DGI Fp2 f_zero_of(const Fp2&) { return fp2_zero(); }
DGI Fp f_one_of(const Fp&) { return fp_one(); }
DGI Fp2 f_one_of(const Fp2&) { return fp2_one(); }

template <class F>
DGI Jac<F> jac_infinity() {
  F z = f_zero_of(F{});
  return Jac<F>{z, z, z};
}
template <class F>
DGI bool jac_is_inf(const Jac<F>& p) {
  return f_is_zero(p.z);
}
template <class F>
DGI Jac<F> jac_from_aff(const Aff<F>& a) {
  if (a.inf) return jac_infinity<F>();
  return Jac<F>{a.x, a.y, f_one_of(F{})};
}
template <class F>
DGI Jac<F> jac_neg(const Jac<F>& p) {
  return Jac<F>{p.x, f_neg(p.y), p.z};
}

// dbl-2009-l (a = 0): 2M + 5S
template <class F>
DGH Jac<F> jac_dbl(const Jac<F>& p) {
  F A = f_sqr(p.x);
  F B = f_sqr(p.y);
  F C = f_sqr(B);
  F D = f_dbl(f_sub(f_sub(f_sqr(f_add(p.x, B)), A), C));
  F E = f_add(f_dbl(A), A);
  F Fv = f_sqr(E);
  F X3 = f_sub(Fv, f_dbl(D));
  F C8 = f_dbl(f_dbl(f_dbl(C)));
  F Y3 = f_sub(f_mul(E, f_sub(D, X3)), C8);
  F Z3 = f_dbl(f_mul(p.y, p.z));
  return Jac<F>{X3, Y3, Z3};  // infinity (z = 0) maps to z = 0
}

// add-2007-bl with the exceptional cases handled
template <class F>
DGH Jac<F> jac_add(const Jac<F>& p, const Jac<F>& q) {
  if (jac_is_inf(p)) return q;
  if (jac_is_inf(q)) return p;
  F Z1Z1 = f_sqr(p.z);
  F Z2Z2 = f_sqr(q.z);
  F U1 = f_mul(p.x, Z2Z2);
  F U2 = f_mul(q.x, Z1Z1);
  F S1 = f_mul(f_mul(p.y, q.z), Z2Z2);
  F S2 = f_mul(f_mul(q.y, p.z), Z1Z1);
  F H = f_sub(U2, U1);
  F r = f_dbl(f_sub(S2, S1));
  if (f_is_zero(H)) {
    if (f_is_zero(r)) return jac_dbl(p);
    return jac_infinity<F>();
  }
  F I = f_sqr(f_dbl(H));
  F J = f_mul(H, I);
  F V = f_mul(U1, I);
  F X3 = f_sub(f_sub(f_sqr(r), J), f_dbl(V));
  F Y3 = f_sub(f_mul(r, f_sub(V, X3)), f_dbl(f_mul(S1, J)));
  F Z3 = f_mul(f_sub(f_sub(f_sqr(f_add(p.z, q.z)), Z1Z1), Z2Z2), H);
  return Jac<F>{X3, Y3, Z3};
}

// madd-2007-bl: q affine (not infinity)
template <class F>
DGH Jac<F> jac_add_aff(const Jac<F>& p, const F& qx, const F& qy) {
  if (jac_is_inf(p)) return Jac<F>{qx, qy, f_one_of(F{})};
  F Z1Z1 = f_sqr(p.z);
  F U2 = f_mul(qx, Z1Z1);
  F S2 = f_mul(f_mul(qy, p.z), Z1Z1);
  F H = f_sub(U2, p.x);
  F r = f_dbl(f_sub(S2, p.y));
  if (f_is_zero(H)) {
    if (f_is_zero(r)) return jac_dbl(p);
    return jac_infinity<F>();
  }
  F HH = f_sqr(H);
  F I = f_dbl(f_dbl(HH));
  F J = f_mul(H, I);
  F V = f_mul(p.x, I);
  F X3 = f_sub(f_sub(f_sqr(r), J), f_dbl(V));
  F Y3 = f_sub(f_mul(r, f_sub(V, X3)), f_dbl(f_mul(p.y, J)));
  F Z3 = f_sub(f_sub(f_sqr(f_add(p.z, H)), Z1Z1), HH);
  return Jac<F>{X3, Y3, Z3};
}

// The same mixed addition for G2 ordered for a small live set (Z3 first, then Z1, Z1Z1 and H, HH die; at most
// about seven Fp2 values live at once) with the exceptional cases (P = +-Q) out of line: the per-point loop of
// the MSM chunk sums keeps its register file free of the doubling formula.  Identical results to jac_add_aff.
DGN G2J g2_add_aff_rare(const G2J& p, const Fp2& qx, const Fp2& qy) { return jac_add_aff(p, qx, qy); }
DGN G2J g2_add_rare(const G2J& p, const G2J& q) { return jac_add(p, q); }
DGI G2J g2_madd_lean(const G2J& p, const Fp2& qx, const Fp2& qy) {
  if (jac_is_inf(p)) return G2J{qx, qy, fp2_one()};
  const Fp2 Z1Z1 = fp2_sqr(p.z);
  const Fp2 H = fp2_sub(fp2_mul(qx, Z1Z1), p.x);
  const Fp2 r = fp2_dbl(fp2_sub(fp2_mul(fp2_mul(qy, p.z), Z1Z1), p.y));
  if (fp2_is_zero(H)) return g2_add_aff_rare(p, qx, qy);
  const Fp2 HH = fp2_sqr(H);
  const Fp2 Z3 = fp2_sub(fp2_sub(fp2_sqr(fp2_add(p.z, H)), Z1Z1), HH);
  const Fp2 I = fp2_dbl(fp2_dbl(HH));
  const Fp2 J = fp2_mul(H, I);
  const Fp2 V = fp2_mul(p.x, I);
  const Fp2 X3 = fp2_sub(fp2_sub(fp2_sqr(r), J), fp2_dbl(V));
  const Fp2 Y3 = fp2_sub(fp2_mul(r, fp2_sub(V, X3)), fp2_dbl(fp2_mul(p.y, J)));
  return G2J{X3, Y3, Z3};
}

// The same mixed addition with the accumulator in LDS (one slot per lane): its nine Fp2 limbs leave the register
// file, which then holds only the formula's temporaries (at most five Fp2 values and one product), so the chunk
// sums run at 2 waves/SIMD without scratch.  Identical results to g2_madd_lean.
#ifndef DG_MADD_FORM
#define DG_MADD_FORM 3  // Fp2 products of g2_madd_lds: 1 one call each (fp2_mul_rc), 2 inlined (fp2_mul_in), 3 inlined and serialised
#endif
#if DG_MADD_FORM == 1
#define DG_MADD_MUL fp2_mul_rc
#define DG_MADD_SQR fp2_sqr_rc
#elif DG_MADD_FORM == 3
#define DG_MADD_MUL fp2_mul_seq
#define DG_MADD_SQR fp2_sqr_seq
#else
#define DG_MADD_MUL fp2_mul_in
#define DG_MADD_SQR fp2_sqr_in
#endif
// dbl-2009-l with the accumulator in LDS, products as g2_madd_lds (the identity stays the identity)
template <class S>
DGI void g2_dbl_lds(S& a) {
  const Fp2 A = DG_MADD_SQR(a.x);
  const Fp2 B = DG_MADD_SQR(a.y);
  const Fp2 C = DG_MADD_SQR(B);
  const Fp2 D = fp2_dbl(fp2_sub(fp2_sub(DG_MADD_SQR(fp2_add(a.x, B)), A), C));
  const Fp2 E = fp2_add(fp2_dbl(A), A);
  a.z = fp2_dbl(DG_MADD_MUL(a.y, a.z));
  const Fp2 X3 = fp2_sub(DG_MADD_SQR(E), fp2_dbl(D));
  a.x = X3;
  a.y = fp2_sub(DG_MADD_MUL(E, fp2_sub(D, X3)), fp2_dbl(fp2_dbl(fp2_dbl(C))));
}

template <class S>
DGI void g2_madd_lds(S& a, const Fp2& qx, const Fp2& qy) {
  if (fp2_is_zero(a.z)) {
    a.x = qx;
    a.y = qy;
    a.z = fp2_one();
    return;
  }
  const Fp2 Z1Z1 = DG_MADD_SQR(a.z);
  const Fp2 H = fp2_sub(DG_MADD_MUL(qx, Z1Z1), a.x);
  const Fp2 r = fp2_dbl(fp2_sub(DG_MADD_MUL(DG_MADD_MUL(qy, a.z), Z1Z1), a.y));
  if (fp2_is_zero(H)) {  // a = +-q: the tangent, or the identity (inline: no call frame in scratch)
    if (fp2_is_zero(r)) g2_dbl_lds(a);
    else a.z = fp2_zero();
    return;
  }
  const Fp2 HH = DG_MADD_SQR(H);
  a.z = fp2_sub(fp2_sub(DG_MADD_SQR(fp2_add(a.z, H)), Z1Z1), HH);
  const Fp2 I = fp2_dbl(fp2_dbl(HH));
  const Fp2 J = DG_MADD_MUL(H, I);
  const Fp2 V = DG_MADD_MUL(a.x, I);
  const Fp2 YJ2 = fp2_dbl(DG_MADD_MUL(a.y, J));
  const Fp2 X3 = fp2_sub(fp2_sub(DG_MADD_SQR(r), J), fp2_dbl(V));
  a.x = X3;
  a.y = fp2_sub(DG_MADD_MUL(r, fp2_sub(V, X3)), YJ2);
}

// The full addition (add-2007-bl) with the accumulator in LDS, products as g2_madd_lds; q any Jacobian point.
// Identical results to jac_add (exceptional cases out of line).
template <class S>
DGI void g2_add_lds(S& a, const G2J& q) {
  if (jac_is_inf(q)) return;
  if (fp2_is_zero(a.z)) {
    a.x = q.x;
    a.y = q.y;
    a.z = q.z;
    return;
  }
  const Fp2 Z1Z1 = DG_MADD_SQR(a.z);
  const Fp2 Z2Z2 = DG_MADD_SQR(q.z);
  const Fp2 U1 = DG_MADD_MUL(a.x, Z2Z2);
  const Fp2 S1 = DG_MADD_MUL(DG_MADD_MUL(a.y, q.z), Z2Z2);
  const Fp2 H = fp2_sub(DG_MADD_MUL(q.x, Z1Z1), U1);
  const Fp2 r = fp2_dbl(fp2_sub(DG_MADD_MUL(DG_MADD_MUL(q.y, a.z), Z1Z1), S1));
  if (fp2_is_zero(H)) {  // a = +-q, as g2_madd_lds
    if (fp2_is_zero(r)) g2_dbl_lds(a);
    else a.z = fp2_zero();
    return;
  }
  a.z = DG_MADD_MUL(fp2_sub(fp2_sub(DG_MADD_SQR(fp2_add(a.z, q.z)), Z1Z1), Z2Z2), H);
  const Fp2 I = DG_MADD_SQR(fp2_dbl(H));
  const Fp2 J = DG_MADD_MUL(H, I);
  const Fp2 V = DG_MADD_MUL(U1, I);
  const Fp2 SJ2 = fp2_dbl(DG_MADD_MUL(S1, J));
  const Fp2 X3 = fp2_sub(fp2_sub(DG_MADD_SQR(r), J), fp2_dbl(V));
  a.x = X3;
  a.y = fp2_sub(DG_MADD_MUL(r, fp2_sub(V, X3)), SJ2);
}

// Affine pair additions with an externally supplied inverse (the affine levels of the MSM, msm.h; Montgomery's
// trick over the batch supplies 1 / N(d)).  kind: 0 pass-through (an identity operand), 1 chord (x1 != x2),
// 2 tangent (P + P), 3 identity result (P + (-P)).  E' has no 2-torsion (h2 is odd), so a tangent has y != 0.
DGI uint32_t g2_aff_kind(const G2A& p, const G2A& q) {
  if (p.inf || q.inf) return 0;
  if (!fp2_eq(p.x, q.x)) return 1;
  return fp2_eq(p.y, q.y) ? 2u : 3u;
}
// N(d) of the pair's denominator d (chord: x2 - x1, tangent: 2 y1); 1 where no inversion is needed
DGI Fp g2_aff_den(const G2A& p, const G2A& q, uint32_t kind) {
  if (kind == 1) return fp2_norm(fp2_sub(q.x, p.x));
  if (kind == 2) return fp2_norm(fp2_dbl(p.y));
  return fp_one();
}
// p + q given nv = 1 / g2_aff_den(p, q, kind): 1/d = conj(d) nv, lambda = (y2 - y1)/d or 3 x1^2 / d,
// x3 = lambda^2 - x1 - x2, y3 = lambda (x1 - x3) - y1 (products serialised, field.h fp2_mul_seq)
DGI G2A g2_aff_sum(const G2A& p, const G2A& q, uint32_t kind, const Fp& nv) {
  if (kind == 0) return p.inf ? q : p;
  if (kind == 3) return G2A{fp2_zero(), fp2_zero(), true};
  const Fp2 d = kind == 1 ? fp2_sub(q.x, p.x) : fp2_dbl(p.y);
  const Fp2 dinv = Fp2{fp_mul_seq(d.c0, nv), fp_neg(fp_mul_seq(d.c1, nv))};
  Fp2 num;
  if (kind == 1) {
    num = fp2_sub(q.y, p.y);
  } else {
    const Fp2 xx = fp2_sqr_seq(p.x);
    num = fp2_add(fp2_dbl(xx), xx);
  }
  const Fp2 lam = fp2_mul_seq(num, dinv);
  const Fp2 x3 = fp2_sub(fp2_sub(fp2_sqr_seq(lam), p.x), q.x);
  return G2A{x3, fp2_sub(fp2_mul_seq(lam, fp2_sub(p.x, x3)), p.y), false};
}

template <class F>
DGH bool jac_eq(const Jac<F>& p, const Jac<F>& q) {
  bool pi = jac_is_inf(p), qi = jac_is_inf(q);
  if (pi || qi) return pi && qi;
  F Z1Z1 = f_sqr(p.z);
  F Z2Z2 = f_sqr(q.z);
  if (!f_eq(f_mul(p.x, Z2Z2), f_mul(q.x, Z1Z1))) return false;
  return f_eq(f_mul(f_mul(p.y, q.z), Z2Z2), f_mul(f_mul(q.y, p.z), Z1Z1));
}

// [k]P for a 64-bit scalar (double-and-add, MSB first); mixed additions when P has Z = 1
template <class F>
DGH Jac<F> jac_mul_u64(const Jac<F>& p, uint64_t k) {
  const bool aff = f_eq(p.z, f_one_of(F{}));
  Jac<F> acc = jac_infinity<F>();
  for (int b = 63; b >= 0; --b) {
    acc = jac_dbl(acc);
    if ((k >> b) & 1) acc = aff ? jac_add_aff(acc, p.x, p.y) : jac_add(acc, p);
  }
  return acc;
}
// [k]P for a 256-bit scalar given as 8 little-endian 32-bit limbs (plain integer)
template <class F>
DGH Jac<F> jac_mul_u256(const Jac<F>& p, const uint32_t* k) {
  Jac<F> acc = jac_infinity<F>();
  // fixed 4-bit window with a 16-entry table would need 16 points in registers; keep double-and-add
  for (int w = 7; w >= 0; --w) {
    uint32_t kw = k[w];
    for (int b = 31; b >= 0; --b) {
      acc = jac_dbl(acc);
      if ((kw >> b) & 1) acc = jac_add(acc, p);
    }
  }
  return acc;
}

template <class F>
DGI Aff<F> jac_to_aff_with_inv(const Jac<F>& p, const F& zinv) {
  F zi2 = f_sqr(zinv);
  return Aff<F>{f_mul(p.x, zi2), f_mul(p.y, f_mul(zi2, zinv)), false};
}
DGH G1A g1_to_aff(const G1J& p) {
  if (jac_is_inf(p)) return G1A{fp_zero(), fp_zero(), true};
  return jac_to_aff_with_inv(p, fp_inv(p.z));
}
DGH G2A g2_to_aff(const G2J& p) {
  if (jac_is_inf(p)) return G2A{fp2_zero(), fp2_zero(), true};
  return jac_to_aff_with_inv(p, fp2_inv(p.z));
}

// ---- G2 endomorphism psi = untwist o Frobenius o twist, subgroup check, cofactor clearing
DGH G2J g2_psi(const G2J& p) {
  return G2J{fp2_mul(fp2_conj(p.x), fp2_const(PSI_CX)), fp2_mul(fp2_conj(p.y), fp2_const(PSI_CY)), fp2_conj(p.z)};
}
// [z]P with z = -Z_ABS
DGI G2J g2_mul_z(const G2J& p) { return jac_neg(jac_mul_u64(p, Z_ABS)); }

// k <- k / d, returns k mod d (k: 8 little-endian 32-bit limbs; bitwise long division, d < 2^64)
DGI uint64_t u256_divmod_u64(uint32_t (&k)[8], uint64_t d) {
  uint64_t rem = 0;
  for (int w = 7; w >= 0; --w) {
    uint32_t q = 0, kw = k[w];
    for (int b = 31; b >= 0; --b) {
      const uint64_t top = rem >> 63;
      rem = (rem << 1) | ((kw >> b) & 1u);
      const bool ge = top || rem >= d;
      rem = ge ? rem - d : rem;  // the true value < 2d, so the wrap is exact
      q |= (ge ? 1u : 0u) << b;
    }
    k[w] = q;
  }
  return rem;
}
// psi on an affine point: (conj(x) cx, conj(y) cy)
DGI void g2_psi_aff(Fp2& x, Fp2& y) {
  x = fp2_mul(fp2_conj(x), fp2_const(PSI_CX));
  y = fp2_mul(fp2_conj(y), fp2_const(PSI_CY));
}
// [k]P for P in G2 (affine) and a plain scalar k < r (8 little-endian limbs).  psi acts on G2 as [z],
// z = -Z_ABS, and r < Z_ABS^4, so with the base-Z_ABS digits k = d0 + d1 Z + d2 Z^2 + d3 Z^3
// (d_i < 2^64):  [k]P = [d0]P + [d1](-psi P) + [d2](psi^2 P) + [d3](-psi^3 P).  Straus over the four
// digits in non-adjacent form: 64 shared doublings and ~86 mixed additions, ~2.5x fewer group
// operations than 255-bit double-and-add (jac_mul_u256).
DGH G2J g2_mul_u256_psi(const G2A& p, const uint32_t* k) {
  if (p.inf) return jac_infinity<Fp2>();
  uint32_t q[8];
  for (int w = 0; w < 8; ++w) q[w] = k[w];
  uint64_t d[4];
  d[0] = u256_divmod_u64(q, Z_ABS);
  d[1] = u256_divmod_u64(q, Z_ABS);
  d[2] = u256_divmod_u64(q, Z_ABS);
  d[3] = (uint64_t)q[1] << 32 | q[0];  // < Z_ABS since k < Z_ABS^4
  // Only P and psi(P) stay live (96 words instead of 192 for the four points: the spills of the scalar
  // loop were a few hundred GB of scratch traffic per 100k-round Recover, PMC): psi^2 is (x, y) -> (w x, -y)
  // on E2 (w = N(PSI_CX), a cube root of unity in Fp), so P_2 = psi^2 P = (w x0, -y0) and
  // P_3 = -psi^3 P = (w x1, y1) cost one Fp2 x Fp product of the x-coordinate where they are added.
  const Fp2 x0 = p.x, y0 = p.y;
  Fp2 x1 = p.x, y1 = p.y;
  g2_psi_aff(x1, y1);
  auto add_i = [&](const G2J& acc, int i, bool neg) {
    const Fp2 x = i == 0 ? x0 : i == 1 ? x1 : fp2_mul_fp(i == 2 ? x0 : x1, fp_const(PSI2_W));
    const Fp2 y = i == 0 ? y0 : i == 1 ? fp2_neg(y1) : i == 2 ? fp2_neg(y0) : y1;
    return jac_add_aff(acc, x, neg ? fp2_neg(y) : y);
  };
  // non-adjacent forms of the digits (65 signed digits, ~1/3 non-zero): h = 3d, digit j = h_{j+1} - d_{j+1}
  uint64_t pos[4], neg[4];
  uint32_t pos64 = 0;
  for (int i = 0; i < 4; ++i) {
    const uint64_t hl = d[i] + (d[i] << 1), hh = (d[i] >> 63) + (hl < d[i] ? 1u : 0u);
    pos[i] = ((hl & ~d[i]) >> 1) | (hh << 63);  // bits 0..63; bit 64 of the form is hh >> 1
    neg[i] = (~hl & d[i]) >> 1;
    pos64 |= (uint32_t)(hh >> 1) << i;
  }
  G2J acc = jac_infinity<Fp2>();
#pragma unroll
  for (int i = 0; i < 4; ++i)
    if ((pos64 >> i) & 1) acc = add_i(acc, i, false);
  for (int b = 63; b >= 0; --b) {
    acc = jac_dbl(acc);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      if ((pos[i] >> b) & 1) acc = add_i(acc, i, false);
      if ((neg[i] >> b) & 1) acc = add_i(acc, i, true);
    }
  }
  return acc;
}
// The same product with the accumulator in LDS (`acc`: one G2JStore slot per lane at the call site,
// hostcheck): doublings and mixed additions as g2_dbl_lds / g2_madd_lds, so the register file holds P,
// psi(P) and one formula's temporaries (the in-register form spills ~740 VGPRs).  Same result.
template <class SJ>
DGI void g2_mul_u256_psi_lds(const G2A& p, const uint32_t* k, SJ& acc) {
  acc.z = fp2_zero();
  if (p.inf) return;
  uint32_t q[8];
  for (int w = 0; w < 8; ++w) q[w] = k[w];
  uint64_t d[4];
  d[0] = u256_divmod_u64(q, Z_ABS);
  d[1] = u256_divmod_u64(q, Z_ABS);
  d[2] = u256_divmod_u64(q, Z_ABS);
  d[3] = (uint64_t)q[1] << 32 | q[0];
  const Fp2 x0 = p.x, y0 = p.y;
  Fp2 x1 = p.x, y1 = p.y;
  g2_psi_aff(x1, y1);
  auto add_i = [&](int i, bool neg) {
    const Fp2 x = i == 0 ? x0 : i == 1 ? x1 : fp2_mul_fp(i == 2 ? x0 : x1, fp_const(PSI2_W));
    const Fp2 y = i == 0 ? y0 : i == 1 ? fp2_neg(y1) : i == 2 ? fp2_neg(y0) : y1;
    g2_madd_lds(acc, x, neg ? fp2_neg(y) : y);
  };
  uint64_t pos[4], neg[4];
  uint32_t pos64 = 0;
  for (int i = 0; i < 4; ++i) {
    const uint64_t hl = d[i] + (d[i] << 1), hh = (d[i] >> 63) + (hl < d[i] ? 1u : 0u);
    pos[i] = ((hl & ~d[i]) >> 1) | (hh << 63);
    neg[i] = (~hl & d[i]) >> 1;
    pos64 |= (uint32_t)(hh >> 1) << i;
  }
#pragma unroll
  for (int i = 0; i < 4; ++i)
    if ((pos64 >> i) & 1) add_i(i, false);
  for (int b = 63; b >= 0; --b) {
    g2_dbl_lds(acc);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      if ((pos[i] >> b) & 1) add_i(i, false);
      if ((neg[i] >> b) & 1) add_i(i, true);
    }
  }
}
// The same product, regular: the four psi digits in the sign-aligned column form of Faz-Hernandez, Longa and
// Sanchez ("Efficient and secure algorithms for GLV-based scalar multiplication", GLV-SAC).  With d0 made odd
// (d0 + 1, corrected by one final subtraction of P), d0 = 2^64 + sum_{j<64} s_j 2^j with s_j = +-1, and every
// other digit d_i = sum_{j<=64} s_j u_ij 2^j with u_ij in {0, 1}: each column is s_j T[u_1j + 2 u_2j + 4 u_3j],
// T[u] = P_0 + u_1 P_1 + u_2 P_2 + u_3 P_3 (8 affine points, one batch inversion).  65 doublings and 65 mixed
// additions whatever the lanes' scalars (a per-bit select of every digit's addition took 64 + 256): the Recover terms of rounds with
// different share sets (divergent waves).  The table is indexed per lane, so it lives in scratch.  P_i are
// multiples [|z|^i]P with 1 + |z| + |z|^2 + |z|^3 < r, so no table entry is the identity or +- another.
DGH G2J g2_mul_u256_psi_sac(const G2A& p, const uint32_t* k) {
  if (p.inf) return jac_infinity<Fp2>();
  uint32_t q[8];
  for (int w = 0; w < 8; ++w) q[w] = k[w];
  uint64_t d[4];
  d[0] = u256_divmod_u64(q, Z_ABS);
  d[1] = u256_divmod_u64(q, Z_ABS);
  d[2] = u256_divmod_u64(q, Z_ABS);
  d[3] = (uint64_t)q[1] << 32 | q[0];
  const bool even = (d[0] & 1) == 0;
  const uint64_t k0 = d[0] + (even ? 1u : 0u);  // < Z_ABS + 1: no overflow
  const uint64_t sgn = k0 >> 1;                  // bit j set: s_j = +1 (j < 64); s_64 = +1
  uint64_t um[3];
  uint32_t top = 0;  // u_{i,64}
  for (int i = 0; i < 3; ++i) {
    uint64_t a = d[i + 1], m = 0;
    for (int j = 0; j < 64; ++j) {
      const uint64_t bit = a & 1u;
      m |= bit << j;
      a = (a >> 1) + (bit & ~(sgn >> j) & 1u);  // b_j = -1: a = (a + 1) / 2
    }
    um[i] = m;
    top |= (uint32_t)a << i;  // a is 0 or 1 here
  }
  // T[u], u = u1 + 2 u2 + 4 u3 (Jacobian, then one inversion of the product of the Z's)
  Fp2 px[4], py[4];
  px[0] = p.x;
  py[0] = p.y;
  for (int i = 1; i < 4; ++i) {
    px[i] = px[i - 1];
    py[i] = py[i - 1];
    g2_psi_aff(px[i], py[i]);
  }
  py[1] = fp2_neg(py[1]);
  py[3] = fp2_neg(py[3]);
  G2J tj[8];
  tj[0] = G2J{px[0], py[0], fp2_one()};
  for (int u = 1; u < 8; ++u) {
    const int hi = u & 4 ? 3 : (u & 2 ? 2 : 1);  // highest set bit of u -> P_hi
    tj[u] = g2_madd_lean(tj[u & ~(1 << (hi - 1))], px[hi], py[hi]);
  }
  Fp2 pref[8];
  pref[0] = fp2_one();
  for (int u = 1; u < 8; ++u) pref[u] = fp2_mul(pref[u - 1], tj[u].z);
  Fp2 inv = fp2_inv(pref[7]);
  G2A tab[8];
  tab[0] = G2A{px[0], py[0], false};
  for (int u = 7; u >= 1; --u) {
    const Fp2 zi = fp2_mul(inv, pref[u - 1]);
    inv = fp2_mul(inv, tj[u].z);
    const Fp2 zi2 = fp2_sqr(zi);
    tab[u] = G2A{fp2_mul(tj[u].x, zi2), fp2_mul(tj[u].y, fp2_mul(zi2, zi)), false};
  }
  G2J acc{tab[top].x, tab[top].y, fp2_one()};
  for (int j = 63; j >= 0; --j) {
    acc = jac_dbl(acc);
    const uint32_t u = (uint32_t)((um[0] >> j) & 1u) | (uint32_t)((um[1] >> j) & 1u) << 1 |
                       (uint32_t)((um[2] >> j) & 1u) << 2;
    const G2A t = tab[u];
    const bool pos = (sgn >> j) & 1u;
    acc = g2_madd_lean(acc, t.x, fp2_sel(pos, fp2_neg(t.y), t.y));  // fp2_sel(c, a, b) = c ? b : a
  }
  const G2J fix = g2_madd_lean(acc, px[0], fp2_neg(py[0]));
  return G2J{fp2_sel(even, acc.x, fix.x), fp2_sel(even, acc.y, fix.y), fp2_sel(even, acc.z, fix.z)};
}
// sum_i [d_i] P_i over four points (any of them may be the identity) and 64-bit digits, by the same
// sign-aligned column form with a Jacobian table (full additions, no inversion, every exceptional case
// handled by jac_add): 65 doublings + 65 additions + 7 for the table, whatever the digits.  The random
// linear combinations of the per-round group tests (kernels.h verify_group), in G1 and in G2.
template <class F>
DGH Jac<F> jac_msm4_sac(const Jac<F>* p, const uint64_t* d) {
  const bool even = (d[0] & 1) == 0;
  const uint64_t k0 = d[0] + (even ? 1u : 0u);  // even d0 <= 2^64 - 2: no overflow
  const uint64_t sgn = k0 >> 1;
  uint64_t um[3];
  uint32_t top = 0;
  for (int i = 0; i < 3; ++i) {
    uint64_t a = d[i + 1], m = 0;
    for (int j = 0; j < 64; ++j) {
      const uint64_t bit = a & 1u;
      m |= bit << j;
      a = (a >> 1) + (bit & ~(sgn >> j) & 1u);
    }
    um[i] = m;
    top |= (uint32_t)a << i;
  }
  Jac<F> tab[8];
  tab[0] = p[0];
  for (int u = 1; u < 8; ++u) {
    const int hi = u & 4 ? 3 : (u & 2 ? 2 : 1);
    tab[u] = jac_add(tab[u & ~(1 << (hi - 1))], p[hi]);
  }
  Jac<F> acc = tab[top];
  for (int j = 63; j >= 0; --j) {
    acc = jac_dbl(acc);
    const uint32_t u = (uint32_t)((um[0] >> j) & 1u) | (uint32_t)((um[1] >> j) & 1u) << 1 |
                       (uint32_t)((um[2] >> j) & 1u) << 2;
    const Jac<F> t = tab[u];
    const bool pos = (sgn >> j) & 1u;
    acc = jac_add(acc, Jac<F>{t.x, f_sel(pos, f_neg(t.y), t.y), t.z});
  }
  const Jac<F> fix = jac_add(acc, jac_neg(p[0]));
  return Jac<F>{f_sel(even, acc.x, fix.x), f_sel(even, acc.y, fix.y), f_sel(even, acc.z, fix.z)};
}
// P in G2  <=>  psi(P) == [z]P   (Scott, "A note on group membership tests for G1, G2 and GT")
DGH bool g2_in_subgroup(const G2J& p) { return jac_eq(g2_psi(p), g2_mul_z(p)); }
// the same test for an affine point (decoded signatures): [|z|]P by double-and-add from the top bit with
// mixed additions (P has Z = 1), psi(P) affine, and a Z1 = 1 comparison
DGH bool g2_in_subgroup_aff(const Fp2& x, const Fp2& y) {
  G2J acc{x, y, fp2_one()};
  for (int b = 62; b >= 0; --b) {
    acc = jac_dbl(acc);
    if ((Z_ABS >> b) & 1) acc = jac_add_aff(acc, x, y);
  }
  // [z]P = -acc; psi(P) = (conj(x) cx, conj(y) cy) affine
  if (jac_is_inf(acc)) return false;  // psi(P) is never the identity for an affine P
  Fp2 px = fp2_mul(fp2_conj(x), fp2_const(PSI_CX)), py = fp2_mul(fp2_conj(y), fp2_const(PSI_CY));
  Fp2 zz = fp2_sqr(acc.z);
  if (!fp2_eq(fp2_mul(px, zz), acc.x)) return false;
  return fp2_eq(fp2_mul(py, fp2_mul(zz, acc.z)), fp2_neg(acc.y));
}
// RFC 9380 Appendix G.3 (Budroni-Pintore): h_eff * P = [z^2 - z - 1]P + [z - 1]psi(P) + psi^2(2P)
DGH G2J g2_clear_cofactor(const G2J& p) {
  G2J t1 = g2_mul_z(p);
  G2J t2 = g2_psi(p);
  G2J t3 = g2_psi(g2_psi(jac_dbl(p)));
  t3 = jac_add(t3, jac_neg(t2));
  t2 = jac_add(t1, t2);
  t2 = g2_mul_z(t2);
  t3 = jac_add(t3, t2);
  t3 = jac_add(t3, jac_neg(t1));
  return jac_add(t3, jac_neg(p));
}
// G1 subgroup check by [r]P == O (keys and commits only: a handful per batch)
DGH bool g1_in_subgroup(const G1J& p) {
  // r as 8 little-endian limbs
  return jac_is_inf(jac_mul_u256(p, R_LIMBS));
}

// ---- ZCash decoding.  Status: 0 ok, 1 = decode error.
DGH bool g1_decompress(G1A& out, const uint8_t* in, bool subgroup_check) {
  uint8_t f = in[0];
  if (!(f & 0x80)) return false;
  if (f & 0x40) {
    if (f != 0xc0) return false;
    uint32_t o = 0;
    for (int i = 1; i < 48; ++i) o |= in[i];
    if (o) return false;
    out = G1A{fp_zero(), fp_zero(), true};
    return true;
  }
  uint8_t b[48];
  for (int i = 0; i < 48; ++i) b[i] = in[i];
  b[0] &= 0x1f;
  Fp x;
  if (!fp_from_be48_plain(x, b)) return false;
  x = fp_to_mont(x);
  Fp rhs = fp_add(fp_mul(fp_sqr(x), x), fp_const(FP_B_G1));
  Fp y;
  if (!fp_sqrt(y, rhs)) return false;
  if (((f & 0x20) != 0) != fp_lex_largest(y)) y = fp_neg(y);
  out = G1A{x, y, false};
  if (subgroup_check && !g1_in_subgroup(jac_from_aff(out))) return false;
  return true;
}
DGH bool g2_decompress(G2A& out, const uint8_t* in, bool subgroup_check) {
  uint8_t f = in[0];
  if (!(f & 0x80)) return false;
  if (f & 0x40) {
    if (f != 0xc0) return false;
    uint32_t o = 0;
    for (int i = 1; i < 96; ++i) o |= in[i];
    if (o) return false;
    out = G2A{fp2_zero(), fp2_zero(), true};
    return true;
  }
  uint8_t b[48];
  for (int i = 0; i < 48; ++i) b[i] = in[i];
  b[0] &= 0x1f;
  Fp x1, x0;
  if (!fp_from_be48_plain(x1, b)) return false;
  if (!fp_from_be48_plain(x0, in + 48)) return false;
  Fp2 x{fp_to_mont(x0), fp_to_mont(x1)};
  Fp2 rhs = fp2_add(fp2_mul(fp2_sqr(x), x), fp2_const(FP2_B_G2));
  Fp2 y;
  if (!fp2_sqrt(y, rhs)) return false;
  if (((f & 0x20) != 0) != fp2_lex_largest(y)) y = fp2_neg(y);
  out = G2A{x, y, false};
  if (subgroup_check && !g2_in_subgroup_aff(x, y)) return false;
  return true;
}
DGI void g1_compress_aff(uint8_t* out, const G1A& a) {
  if (a.inf) {
    out[0] = 0xc0;
    for (int i = 1; i < 48; ++i) out[i] = 0;
    return;
  }
  fp_to_be48(out, a.x);
  out[0] |= 0x80;
  if (fp_lex_largest(a.y)) out[0] |= 0x20;
}
DGI void g2_compress_aff(uint8_t* out, const G2A& a) {
  if (a.inf) {
    out[0] = 0xc0;
    for (int i = 1; i < 96; ++i) out[i] = 0;
    return;
  }
  fp_to_be48(out, a.x.c1);
  fp_to_be48(out + 48, a.x.c0);
  out[0] |= 0x80;
  if (fp2_lex_largest(a.y)) out[0] |= 0x20;
}

}  // namespace dg
