// Two-lane teams for the per-item pairing checks (A4 / A5 on single shares and on Recover's group tests).
//
// One lane holding a whole Fp12 (576 B) and the chain of the final exponentiation spilled ~14.5 KB per lane to
// scratch (1.6 TB/s of scratch traffic, 0.16 of the MAC peak).  Here the two lanes 2j, 2j+1 of a
// wave share one check: GT = Fp6[w]/(w^2 - v), f = f0 + f1 w, and lane h holds f_h (one Fp6, 72 words).  Every
// GT operation is written so that both lanes run the same instructions on their own halves (no divergence), and
// the halves cross between the two lanes by DPP (quad_perm 1,0,3,2: a full-rate VALU move, no LDS):
//   f^2          lane 0: (a0 + a1)(a0 + v a1), lane 1: a0 a1 -> one Fp6 product each (complex squaring)
//   f g          lane 0: a0 b0 + v a1 b1,      lane 1: a1 b0 + a0 b1 -> two Fp6 products each
//   f l (line)   l = (c0 + c1 v) + (c4 v) w:   both lanes f_h (c0 + c1 v) + [v] f_{1-h} c4 v -> 8 Fp2 products each
//   cyclotomic   Granger-Scott over the three Fp4 pieces, which straddle the halves: 5 Fp2 squarings per lane
// In the Miller loop each lane owns one of the check's two pairs (its G2 point, line and evaluation); the two
// lines of a step are multiplied into f one after the other.
#pragma once
#include "coop.h"

// The GT building blocks (t2_sqr, t2_mul, t2_mul_line, t2_cyc_sqr, t2_frob) are out of line (DG_T2_BLOCK): inlined
// into the loops, the verify TU took 7.5 minutes to build and its private segment grew (13.0 -> 18.3 KB per lane).
#ifndef DG_T2_BLOCK
#define DG_T2_BLOCK DG12
#endif

namespace dg {

#if defined(__HIP_DEVICE_COMPILE__)
DGI uint32_t t2_x(uint32_t v) { return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, false); }
#else
// host builds: the test harness (tests/native/hostcheck.cpp) runs a team as two threads and exchanges through this
// hook; without it a host build is a team of one
inline thread_local uint32_t (*g_t2_xchg)(uint32_t) = nullptr;
DGI uint32_t t2_x(uint32_t v) { return g_t2_xchg ? g_t2_xchg(v) : v; }
#endif
DGI Fp t2_x(const Fp& a) {
  Fp r;
#pragma unroll
  for (int i = 0; i < 12; ++i) r.l[i] = t2_x(a.l[i]);
  return r;
}
DGI Fp2 t2_x(const Fp2& a) { return Fp2{t2_x(a.c0), t2_x(a.c1)}; }
DGI Fp6 t2_x(const Fp6& a) { return Fp6{t2_x(a.c0), t2_x(a.c1), t2_x(a.c2)}; }

DGI Fp6 fp6_one() { return Fp6{fp2_one(), fp2_zero(), fp2_zero()}; }
DGI Fp6 fp6_dbl(const Fp6& a) { return fp6_add(a, a); }
// c ? a : b (the field.h selects take the other order: fp_sel(c, a, b) = c ? b : a)
DGI Fp2 fp2_pick(bool c, const Fp2& a, const Fp2& b) { return fp2_sel(c, b, a); }
DGI Fp6 fp6_pick(bool c, const Fp6& a, const Fp6& b) {
  return Fp6{fp2_pick(c, a.c0, b.c0), fp2_pick(c, a.c1, b.c1), fp2_pick(c, a.c2, b.c2)};
}
DGI bool fp6_is_zero(const Fp6& a) { return fp2_is_zero(a.c0) && fp2_is_zero(a.c1) && fp2_is_zero(a.c2); }

// f^2 (complex squaring: c0 = (a0 + a1)(a0 + v a1) - t - v t, c1 = 2 t, t = a0 a1)
DG_T2_BLOCK Fp6 t2_sqr(const Fp6& F, uint32_t h) {
  const Fp6 O = t2_x(F);
  const Fp6 x = fp6_pick(h, F, fp6_add(F, O));
  const Fp6 y = fp6_pick(h, O, fp6_add(F, fp6_mul_v(O)));
  const Fp6 m = fp6_mul(x, y);
  const Fp6 t = t2_x(m);
  return fp6_pick(h, fp6_dbl(m), fp6_sub(fp6_sub(m, t), fp6_mul_v(t)));
}
// f g (schoolbook over w: each lane's own output half, no exchange of products)
DG_T2_BLOCK Fp6 t2_mul(const Fp6& F, const Fp6& G, uint32_t h) {
  const Fp6 O = t2_x(F), Og = t2_x(G);
  const Fp6 m1 = fp6_mul(F, fp6_pick(h, Og, G));  // lane 0: a0 b0, lane 1: a1 b0
  const Fp6 m2 = fp6_mul(O, fp6_pick(h, G, Og));  // lane 0: a1 b1, lane 1: a0 b1
  return fp6_add(m1, fp6_pick(h, m2, fp6_mul_v(m2)));
}
// f l, l = c0 + c1 v + c4 v w (the line of pairing.h; the same c0, c1, c4 on both lanes)
DG_T2_BLOCK Fp6 t2_mul_line(const Fp6& F, const Fp2& c0, const Fp2& c1, const Fp2& c4, uint32_t h) {
  const Fp6 m = fp6_mul_1(t2_x(F), c4);
  const Fp6 a = fp6_mul_01(F, c0, c1);
  return fp6_add(a, fp6_pick(h, m, fp6_mul_v(m)));
}
DGI Fp6 t2_conj(const Fp6& F, uint32_t h) { return fp6_pick(h, fp6_neg(F), F); }
// f^p: coefficient-wise conj and the Frobenius constants (lane 0: 1, g1, g2; lane 1: d, d g1, d g2)
DG_T2_BLOCK Fp6 t2_frob(const Fp6& F, uint32_t h) {
  const Fp2 g1 = fp2_const(FROB_G1), g2 = fp2_const(FROB_G2), d = fp2_const(FROB_D);
  const Fp2 k0 = fp2_pick(h, d, fp2_one());
  const Fp2 k1 = fp2_pick(h, fp2_mul(d, g1), g1);
  const Fp2 k2 = fp2_pick(h, fp2_mul(d, g2), g2);
  return Fp6{fp2_mul(fp2_conj(F.c0), k0), fp2_mul(fp2_conj(F.c1), k1), fp2_mul(fp2_conj(F.c2), k2)};
}
// f^-1 = (f0 - f1 w) / (f0^2 - v f1^2); the Fp6 inversion on both lanes
DG12 Fp6 t2_inv(const Fp6& F, uint32_t h) {
  const Fp6 s = fp6_sqr(F);
  const Fp6 so = t2_x(s);
  const Fp6 d = fp6_pick(h, fp6_sub(so, fp6_mul_v(s)), fp6_sub(s, fp6_mul_v(so)));
  const Fp6 r = fp6_mul(F, fp6_inv(d));
  return fp6_pick(h, fp6_neg(r), r);
}
// Granger-Scott cyclotomic squaring (field.h fp12_cyc_sqr).  Lane 0 holds (z0, z4, z3), lane 1 (z2, z1, z5); the
// Fp4 pieces (z0, z1), (z2, z3), (z4, z5) straddle the lanes.  Each lane squares its own three coefficients and
// two sums; lane 0 forms the pieces' first components (xi b^2 + a^2), lane 1 the second ((a + b)^2 - a^2 - b^2).
DG_T2_BLOCK Fp6 t2_cyc_sqr(const Fp6& F, uint32_t h) {
  const Fp6 P = t2_x(F);
  const Fp2 q0 = fp2_sqr(F.c0), q1 = fp2_sqr(F.c1), q2 = fp2_sqr(F.c2);
  // lane 0: (z0 + z1)^2, (z4 + z5)^2 (unused);  lane 1: (z2 + z3)^2, (z4 + z5)^2
  const Fp2 x1 = fp2_sqr(fp2_add(F.c0, fp2_pick(h, P.c2, P.c1)));
  const Fp2 x2 = fp2_sqr(fp2_pick(h, fp2_add(P.c1, F.c2), fp2_add(F.c1, P.c2)));
  const Fp2 pq0 = t2_x(q0), pq1 = t2_x(q1), pq2 = t2_x(q2), px1 = t2_x(x1);
  // lane 0: new (z0, z4, z3) = 3 t - 2 z
  const Fp2 a0 = fp2_add(fp2_mul_xi(pq1), q0);  // (z0, z1) first component
  const Fp2 a1 = fp2_add(fp2_mul_xi(q2), pq0);  // (z2, z3)
  const Fp2 a2 = fp2_add(fp2_mul_xi(pq2), q1);  // (z4, z5)
  const Fp6 n0{fp2_sub(fp2_triple(a0), fp2_dbl(F.c0)), fp2_sub(fp2_triple(a1), fp2_dbl(F.c1)),
               fp2_sub(fp2_triple(a2), fp2_dbl(F.c2))};
  // lane 1: new z2 = 3 xi t3 + 2 z2, z1 = 3 t1 + 2 z1, z5 = 3 t1' + 2 z5
  const Fp2 b1 = fp2_sub(fp2_sub(px1, pq0), q1);  // (z0, z1) second component
  const Fp2 b2 = fp2_sub(fp2_sub(x1, q0), pq2);   // (z2, z3)
  const Fp2 b3 = fp2_sub(fp2_sub(x2, pq1), q2);   // (z4, z5)
  const Fp6 n1{fp2_add(fp2_triple(fp2_mul_xi(b3)), fp2_dbl(F.c0)), fp2_add(fp2_triple(b1), fp2_dbl(F.c1)),
               fp2_add(fp2_triple(b2), fp2_dbl(F.c2))};
  return fp6_pick(h, n1, n0);
}
// f == 1 on both lanes of the team
DGI bool t2_is_one(const Fp6& F, uint32_t h) {
  const bool mine = h ? fp6_is_zero(F) : (fp2_eq(F.c0, fp2_one()) && fp2_is_zero(F.c1) && fp2_is_zero(F.c2));
  return mine && t2_x((uint32_t)mine) != 0u;
}
// ---- Looped forms for the hot loops.  An out-of-line Fp or Fp6 routine costs the call ABI at every product
// (operands marshalled into v0..v23, the caller's live set kept in the ~112 callee-saved VGPRs or spilled around the
// call, Fp6 arguments and results through the stack): ~700 instructions of glue per product in t2_exp_z.  Here one
// inlined Fp2 product sits in a loop body, the operands picked and the result accumulated by a switch on the
// (wave-uniform) step: no calls, one copy of the product code, the state in registers.
DGI Fp2 fp2_mul_xi_neg(const Fp2& a) { return fp2_neg(fp2_mul_xi(a)); }
// a b (Karatsuba as field.h fp6_mul: v0..v5, each product accumulated into the outputs at once)
DGI Fp6 fp6_mul_lp(const Fp6& a, const Fp6& b) {
  const Fp2 a12 = fp2_add(a.c1, a.c2), a01 = fp2_add(a.c0, a.c1), a02 = fp2_add(a.c0, a.c2);
  const Fp2 b12 = fp2_add(b.c1, b.c2), b01 = fp2_add(b.c0, b.c1), b02 = fp2_add(b.c0, b.c2);
  Fp2 c0 = fp2_zero(), c1 = fp2_zero(), c2 = fp2_zero();
#pragma nounroll
  for (int j = 0; j < 6; ++j) {
    Fp2 x, y;
    switch (j) {
      case 0: x = a.c0; y = b.c0; break;
      case 1: x = a.c1; y = b.c1; break;
      case 2: x = a.c2; y = b.c2; break;
      case 3: x = a12; y = b12; break;
      case 4: x = a01; y = b01; break;
      default: x = a02; y = b02; break;
    }
    const Fp2 v = fp2_mul_in(x, y);
    switch (j) {
      case 0: c0 = fp2_add(c0, v); c1 = fp2_sub(c1, v); c2 = fp2_sub(c2, v); break;        // v0
      case 1: c0 = fp2_add(c0, fp2_mul_xi_neg(v)); c1 = fp2_sub(c1, v); c2 = fp2_add(c2, v); break;  // v1
      case 2: c0 = fp2_add(c0, fp2_mul_xi_neg(v)); c1 = fp2_add(c1, fp2_mul_xi(v)); c2 = fp2_sub(c2, v); break;
      case 3: c0 = fp2_add(c0, fp2_mul_xi(v)); break;
      case 4: c1 = fp2_add(c1, v); break;
      default: c2 = fp2_add(c2, v); break;
    }
  }
  return Fp6{c0, c1, c2};
}
// f g (t2_mul)
DGI Fp6 t2_mul_lp(const Fp6& F, const Fp6& G, uint32_t h) {
  const Fp6 Og = t2_x(G);
  const Fp6 m1 = fp6_mul_lp(F, fp6_pick(h, Og, G));  // lane 0: a0 b0, lane 1: a1 b0
  const Fp6 O = t2_x(F);
  const Fp6 m2 = fp6_mul_lp(O, fp6_pick(h, G, Og));  // lane 0: a1 b1, lane 1: a0 b1
  return fp6_add(m1, fp6_pick(h, m2, fp6_mul_v(m2)));
}
// cyclotomic squaring (t2_cyc_sqr), the five Fp2 squarings in a loop
DGI Fp6 t2_cyc_sqr_lp(const Fp6& F, uint32_t h) {
  const Fp6 P = t2_x(F);
  const Fp2 s1 = fp2_add(F.c0, fp2_pick(h, P.c2, P.c1));
  const Fp2 s2 = fp2_pick(h, fp2_add(P.c1, F.c2), fp2_add(F.c1, P.c2));
  Fp2 q0, q1, q2, x1, x2;
#pragma nounroll
  for (int j = 0; j < 5; ++j) {
    Fp2 x;
    switch (j) {
      case 0: x = F.c0; break;
      case 1: x = F.c1; break;
      case 2: x = F.c2; break;
      case 3: x = s1; break;
      default: x = s2; break;
    }
    const Fp m = fp_mul_inl(x.c0, x.c1);
    const Fp2 v{fp_mul_inl(fp_add(x.c0, x.c1), fp_sub(x.c0, x.c1)), fp_dbl(m)};
    switch (j) {
      case 0: q0 = v; break;
      case 1: q1 = v; break;
      case 2: q2 = v; break;
      case 3: x1 = v; break;
      default: x2 = v; break;
    }
  }
  const Fp2 pq0 = t2_x(q0), pq1 = t2_x(q1), pq2 = t2_x(q2), px1 = t2_x(x1);
  const Fp2 a0 = fp2_add(fp2_mul_xi(pq1), q0), a1 = fp2_add(fp2_mul_xi(q2), pq0), a2 = fp2_add(fp2_mul_xi(pq2), q1);
  const Fp6 n0{fp2_sub(fp2_triple(a0), fp2_dbl(F.c0)), fp2_sub(fp2_triple(a1), fp2_dbl(F.c1)),
               fp2_sub(fp2_triple(a2), fp2_dbl(F.c2))};
  const Fp2 b1 = fp2_sub(fp2_sub(px1, pq0), q1), b2 = fp2_sub(fp2_sub(x1, q0), pq2), b3 = fp2_sub(fp2_sub(x2, pq1), q2);
  const Fp6 n1{fp2_add(fp2_triple(fp2_mul_xi(b3)), fp2_dbl(F.c0)), fp2_add(fp2_triple(b1), fp2_dbl(F.c1)),
               fp2_add(fp2_triple(b2), fp2_dbl(F.c2))};
  return fp6_pick(h, n1, n0);
}
// a^z, z = -|z| (a in the cyclotomic subgroup: a^-1 = conj(a)).  DG_T2_LOOPED=1: the looped forms (measured
// slower: the loop bodies spill, C5 per-item pass 117 -> 132 ms per launch)
#ifndef DG_T2_LOOPED
#define DG_T2_LOOPED 0
#endif
DG12 Fp6 t2_exp_z(const Fp6& A, uint32_t h) {
  Fp6 acc = A;
  for (int b = 62; b >= 0; --b) {
#if DG_T2_LOOPED
    acc = t2_cyc_sqr_lp(acc, h);
    if ((Z_ABS >> b) & 1) acc = t2_mul_lp(acc, A, h);
#else
    acc = t2_cyc_sqr(acc, h);
    if ((Z_ABS >> b) & 1) acc = t2_mul(acc, A, h);
#endif
  }
  return t2_conj(acc, h);
}
// f^(3 (p^12 - 1) / r) == 1: the chain of pairing.h final_exp_cubed, the last product compared instead of formed
// (b c == 1 <=> b == conj(c) in the cyclotomic subgroup)
DG12 bool t2_final_exp_is_one(const Fp6& F, uint32_t h) {
  const Fp6 f1 = t2_mul(t2_conj(F, h), t2_inv(F, h), h);   // f^(p^6 - 1)
  const Fp6 f2 = t2_mul(t2_frob(t2_frob(f1, h), h), f1, h);  // ^(p^2 + 1)
  const Fp6 c = t2_mul(t2_cyc_sqr(f2, h), f2, h);           // f2^3
  const Fp6 t0 = t2_mul(t2_exp_z(f2, h), t2_conj(f2, h), h);
  const Fp6 t1 = t2_mul(t2_exp_z(t0, h), t2_conj(t0, h), h);
  const Fp6 a = t2_mul(t2_exp_z(t1, h), t2_frob(t1, h), h);
  Fp6 b = t2_mul(t2_exp_z(t2_exp_z(a, h), h), t2_frob(t2_frob(a, h), h), h);
  b = t2_mul(b, t2_conj(a, h), h);
  const Fp6 cc = t2_conj(c, h);
  const bool mine = fp2_eq(b.c0, cc.c0) && fp2_eq(b.c1, cc.c1) && fp2_eq(b.c2, cc.c2);
  return mine && t2_x((uint32_t)mine) != 0u;
}
// multiply f by both lanes' lines of this step: lane 0's first, then lane 1's
DGI Fp6 t2_mul_lines(Fp6 F, const Fp2& c0, const Fp2& c1, const Fp2& c4, uint32_t h) {
  const Fp2 o0 = t2_x(c0), o1 = t2_x(c1), o4 = t2_x(c4);
  F = t2_mul_line(F, fp2_pick(h, o0, c0), fp2_pick(h, o1, c1), fp2_pick(h, o4, c4), h);
  return t2_mul_line(F, fp2_pick(h, c0, o0), fp2_pick(h, c1, o1), fp2_pick(h, c4, o4), h);
}
// Miller loop of the team's two pairs: lane h brings (P, Q) (affine, neither at infinity when `present`; an absent
// pair contributes the line 1 at every step).  Returns the lane's half of prod_h f_{z,Q_h}(P_h), conjugated (z < 0).
DG12 Fp6 t2_miller(const G1A& P, const G2A& Q, bool present, uint32_t h) {
  G2Proj T{Q.x, Q.y, fp2_one()};
  Fp6 F = fp6_pick(h, fp6_zero(), fp6_one());
  for (int b = 62; b >= 0; --b) {
    F = t2_sqr(F, h);
    Fp2 c0, c1, c4;
    line_dbl(T, c0, c1, c4, P.x, P.y);
    F = t2_mul_lines(F, fp2_pick(present, c0, fp2_one()), fp2_pick(present, c1, fp2_zero()),
                     fp2_pick(present, c4, fp2_zero()), h);
    if ((Z_ABS >> b) & 1) {
      line_add(T, Q.x, Q.y, c0, c1, c4, P.x, P.y);
      F = t2_mul_lines(F, fp2_pick(present, c0, fp2_one()), fp2_pick(present, c1, fp2_zero()),
                       fp2_pick(present, c4, fp2_zero()), h);
    }
  }
  return t2_conj(F, h);
}
// the team's pairing check prod_h e(P_h, Q_h) == 1 (kyber's bls.Verify equation with P_1 = -g1)
DGN bool t2_pair_check(const G1A& P, const G2A& Q, bool present, uint32_t h) {
  return t2_final_exp_is_one(t2_miller(P, Q, present, h), h);
}

}  // namespace dg
