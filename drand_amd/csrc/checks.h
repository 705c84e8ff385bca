// Recover's per-item pass (kernels.h verify_group: e(sum rho_i X_i, H_r) == e(g1, sum rho_i S_i))
// as a pipeline of short kernels with HBM-resident state between them, in place of one lane running a whole pairing
// check (k_verify_groups: 512 VGPRs and ~15 KB of scratch per lane, the stack frames of its out-of-line Fp12 calls;
// ~110 GB of scratch traffic per launch).  The kernels are compiled in translation units of their own
// (kernels_check*.hip: DG_FP_CALL=3, DG_INLINE12=1) with every field product inlined and serialised, so each kernel's
// live set is its own few field elements -- no calls, no scratch -- and every loop body holds one call site of each
// formula (loops are not unrolled), so each kernel stays a few tens of thousands of instructions.
//
// The reference's re-verification of t shares against one message (beacon/beacon.go:488) pairs every check of a
// round against the same H_r = h_eff(Q_r): its Miller-loop line coefficients are computed ONCE per round
// (k_ck_round_lines: 68 lines of 3 Fp2, without the G1 point) and every check only evaluates them at its own
// a = sum rho_i X_i (two Fp2 x Fp products per line) -- `north_star`'s precomputed line coefficients.
//
//   per round (once per Recover call):  k_ck_round_lines  H_r = h_eff(Q_r) and its 68 lines RL[s][r]
//   per pass and chunk of checks (G lanes, drand_gpu.hip check_chunk):
//     k_ck_sub       one lane per member: the G2 subgroup check of S_i (accumulator in LDS)
//     k_ck_prep      the group's members: a = sum rho X, b = sum rho S (kernels.h group_combine)
//     k_ck_lines2    the 68 lines of the pair (-g1, b) -> L2[s][g] (b's G2 state lives only here)
//     k_ck_miller    f = the product of both pairs' lines at a and at -g1 (the Fp12 accumulator and one line)
//     k_ck_easy      the easy part f2 = f1 frob^2(f1), f1 = f^-1 conj(f), with the one Fp inversion in the lane
//     5 x [k_ck_expsq2  63 compressed cyclotomic squarings (Karabina, two lanes per check): the 6 powers, their
//                       denominators' norms
//          k_ck_expdec  the 6 norms inverted in the lane (Montgomery's trick, one Fp inversion), decompression, the
//                       product x^z, times the hard part's next factor  (k_ck_explain: the uncompressed chain where
//                       a denominator is zero, same next factor)]
//     k_ck_final     the last factors and == 1 -> good[g];  k_ck_verdict: the members' verdicts.
// Every kernel after the lines is one lane per check with no exchange between lanes (no batch inversion), so a launch
// may be sized for more checks than it holds: `gcnt` (device) gates the lanes on the count a producer reached
// (xr.h: the cross-round isolation of a failed single-key batch launches every level for its worst case).
// Every value equals the one pair_check computes (pairing.h miller_loop, final_exp_cubed, cyc_exp_z): the same
// formulas in the same order, only split across kernels (tests/test_host_arith.py runs the pipeline's pieces on the
// host against pair_check).
#pragma once
#include "fpd.h"

namespace dg {

// minimum waves per SIMD of the pipeline kernels (A/B knob: 1 lets a kernel use the whole 512-entry register file)
#ifndef DG_CK_WAVES
#define DG_CK_WAVES 1
#endif
// ... of the kernels with a smaller live set (k_ck_prep, k_ck_fe1, k_ck_expsq2: measured faster at 2 than at 1, their
// few spills notwithstanding; the Fp12-product kernels lost at 2)
#ifndef DG_CK_WAVES2
#define DG_CK_WAVES2 2
#endif
// ... of k_ck_lines2 / k_ck_round_lines (a G2 point and one line live)
#ifndef DG_CK_L2_WAVES
#define DG_CK_L2_WAVES 1
#endif
// ... of k_ck_sub (its accumulator in LDS: 18 KB per 64-lane workgroup, so at most 2 per SIMD anyway)
#ifndef DG_CK_SUB_WAVES
#define DG_CK_SUB_WAVES 2
#endif
constexpr uint32_t CK_STEPS = 68;      // Miller steps over |z| = 0xd201000000010000: 63 doublings + 5 additions
constexpr uint32_t CK_CHUNK = 524288;  // checks per pipeline launch at most (~45 KB of workspace per check)
constexpr uint32_t CK_NEXP = 5;        // x^z chains of the hard part (one k_ck_explain work list each)
constexpr int CK_NPOW = 6;             // set bits of |z|: the powers a^(2^k) of the compressed chain
constexpr uint32_t CK_GRP = 4;         // members per check at most (kernels.h GRP)

// one Miller-loop line without its G1 point: l = c0 + (c1 P.x) v + (c4 P.y) v w (pairing.h line_dbl / line_add)
struct CkLine {
  Fp2 c0, c1, c4;
};
// a lane past the checks of a launch: g >= G (the host's bound) or, when the device count gcnt is given, g >= *gcnt
DGI bool ck_dead(uint32_t g, uint32_t G, const uint32_t* gcnt) { return g >= G || (gcnt && g >= *gcnt); }
// one check: up to GRP shares of one round (or one share alone)
struct CkState {
  G1AStore a;          // sum rho_i X_i (a single share: its key)
  G2AStore b;          // sum rho_i S_i (a single share: its sigma)
  uint32_t round, np;  // np bit 0: pair (a, H_r) present; bit 1: pair (-g1, b) present (pair_check drops identities)
  uint32_t n, nl;      // members listed, members live (not rejected by the subgroup check)
  uint32_t live[CK_GRP];  // the live members' item indices
};

// pairing.h line_dbl / line_add with c1, c4 left unscaled by P (T: a G2Proj, or an LDS slot with the same x, y, z)
template <class P>
DGI void ck_line_dbl(P& T, CkLine& l) {
  const Fp2 a = fp2_mul_fp(fp2_mul(T.x, T.y), fp_const(FP_TWO_INV));
  const Fp2 b = fp2_sqr(T.y);
  const Fp2 c = fp2_sqr(T.z);
  const Fp2 e = fp2_mul(fp2_const(FP2_B3_G2), c);
  const Fp2 f = fp2_add(fp2_dbl(e), e);
  const Fp2 g = fp2_mul_fp(fp2_add(b, f), fp_const(FP_TWO_INV));
  const Fp2 h = fp2_sub(fp2_sub(fp2_sqr(fp2_add(T.y, T.z)), b), c);
  const Fp2 j = fp2_sqr(T.x);
  l.c0 = fp2_sub(e, b);
  l.c1 = fp2_add(fp2_dbl(j), j);
  l.c4 = fp2_neg(h);
  const Fp2 e2 = fp2_sqr(e);
  T.x = fp2_mul(a, fp2_sub(b, f));
  T.y = fp2_sub(fp2_sqr(g), fp2_add(fp2_dbl(e2), e2));
  T.z = fp2_mul(b, h);
}
template <class P>
DGI void ck_line_add(P& T, const Fp2& qx, const Fp2& qy, CkLine& l) {
  const Fp2 theta = fp2_sub(T.y, fp2_mul(qy, T.z));
  const Fp2 lambda = fp2_sub(T.x, fp2_mul(qx, T.z));
  const Fp2 c = fp2_sqr(theta);
  const Fp2 d = fp2_sqr(lambda);
  const Fp2 e = fp2_mul(lambda, d);
  const Fp2 f = fp2_mul(T.z, c);
  const Fp2 g = fp2_mul(T.x, d);
  const Fp2 h = fp2_sub(fp2_add(e, f), fp2_dbl(g));
  const Fp2 ny = fp2_sub(fp2_mul(theta, fp2_sub(g, h)), fp2_mul(e, T.y));
  T.x = fp2_mul(lambda, h);
  T.y = ny;
  T.z = fp2_mul(T.z, e);
  l.c0 = fp2_sub(fp2_mul(theta, qx), fp2_mul(lambda, qy));
  l.c1 = fp2_neg(theta);
  l.c4 = lambda;
}
// the kind of Miller step s (0..67): a doubling, or the addition after the doubling of a set bit of |z| (scalar)
DGI bool ck_step_is_dbl(uint32_t step) {
  uint32_t s = 0;
  for (int b = 62; b >= 0; --b) {
    if (s++ == step) return true;
    if ((Z_ABS >> b) & 1 && s++ == step) return false;
  }
  return true;
}
// the 68 lines of Q (affine, not the identity) in step order: out(s, line)
template <class Out>
DGI void ck_lines(const Fp2& qx, const Fp2& qy, Out out) {
  G2Proj T{qx, qy, fp2_one()};
#pragma unroll 1
  for (uint32_t s = 0; s < CK_STEPS; ++s) {
    CkLine l;
    if (ck_step_is_dbl(s))
      ck_line_dbl(T, l);
    else
      ck_line_add(T, qx, qy, l);
    out(s, l);
  }
}
// the Miller value of both pairs from their lines (line(s, pair): pair 0 = (a, H_r) at (ax, ay), pair 1 = (-g1, b)),
// conjugated (z < 0): miller_loop<2> of pairing.h step for step -- per step the squaring (not before the first),
// then pair 0's line, then pair 1's
template <class Line>
DGI Fp12 ck_miller(uint32_t np, const Fp& ax, const Fp& ay, Line line) {
  Fp12 f = fp12_one();
  if (!np) return f;
  const Fp gx = fp_const(G1_GEN_X), gy = fp_const(G1_GEN_NEG_Y);
#pragma unroll 1
  for (uint32_t it = 0; it < 2 * CK_STEPS; ++it) {
    const uint32_t s = it >> 1, pair = it & 1;
    if (pair == 0 && s != 0 && ck_step_is_dbl(s)) f = fp12_sqr(f);
    if ((np >> pair) & 1) {
      const CkLine l = line(s, pair);
      const Fp px = fp_sel(pair != 0, ax, gx), py = fp_sel(pair != 0, ay, gy);  // fp_sel(c, a, b) = c ? b : a
      f = fp12_mul_014(f, l.c0, fp2_mul_fp(l.c1, px), fp2_mul_fp(l.c4, py));
    }
  }
  return fp12_conj(f);
}

// ck_miller with the accumulator and the line values in digit form through the whole loop (fpd.h), the accumulator in a
// column outside the register file (Fd12Col: k_ck_miller's LDS): the lines converted as they are read, the accumulator
// back once at the end -- the same value (tests/native/hostcheck.cpp, the digit-form bounds asserted).  17 spilled
// VGPRs against 36 for ck_miller and 213-430 for the digit form with the accumulator in registers; 1% faster than
// ck_miller (k_ck_miller 24.1 -> 23.8 ms per C5 launch)
template <class Line, class C>
DGI Fp12 ck_miller_col(uint32_t np, const Fp& ax, const Fp& ay, Line line, C& f) {
  if (!np) return fp12_one();
  const Fp gx = fp_const(G1_GEN_X), gy = fp_const(G1_GEN_NEG_Y);
  f.set_one();
#pragma unroll 1
  for (uint32_t it = 0; it < 2 * CK_STEPS; ++it) {
    const uint32_t s = it >> 1, pair = it & 1;
    if (pair == 0 && s != 0 && ck_step_is_dbl(s)) fd12_sqr_col(f);
    if ((np >> pair) & 1) {
      const CkLine l = line(s, pair);
      const Fd px = fd_from(fp_sel(pair != 0, ax, gx)), py = fd_from(fp_sel(pair != 0, ay, gy));
      fd12_mul_014_col(f, fd2_from(l.c0), fd2_mul_fp(fd2_from(l.c1), px), fd2_mul_fp(fd2_from(l.c4), py));
    }
  }
  return fp12_conj(f.to_fp12());
}
// the Miller value of ONE pair of a check (pair 0: (a, H) at P = (px, py); pair 1: (-g1, b)), its own squarings included:
// the two pairs' values multiply to ck_miller's (squaring is multiplicative), conjugated.  Two lanes per check halve the
// lane's chain where the checks of a launch are too few to fill the chip (the cross-round isolation, xr.h).
template <class Line>
DGI Fp12 ck_miller1(const Fp& px, const Fp& py, Line line) {
  Fp12 f = fp12_one();
#pragma unroll 1
  for (uint32_t s = 0; s < CK_STEPS; ++s) {
    if (s != 0 && ck_step_is_dbl(s)) f = fp12_sqr(f);
    const CkLine l = line(s);
    f = fp12_mul_014(f, l.c0, fp2_mul_fp(l.c1, px), fp2_mul_fp(l.c4, py));
  }
  return fp12_conj(f);
}

// ck_miller1 with the pair's lines computed in the lane from Q (affine, not the identity) as the loop runs: no line table.
// The isolation's checks (xr.h k_xg_miller) have no per-round line sharing, so storing each check's 68 lines to HBM
// for a second kernel bought nothing but 19.6 KB per pair of workspace and a launch
// (T: the running point's storage, an LDS slot on the device -- out of the register file beside the Fp12 accumulator;
// q(): Q again, for the five addition steps, instead of keeping it live)
template <class LoadQ, class Slot>
DGI Fp12 ck_miller1_fly(LoadQ q, const Fp& px, const Fp& py, Slot& T) {
  {
    const G2A q0 = q();
    T.x = q0.x;
    T.y = q0.y;
    T.z = fp2_one();
  }
  Fp12 f = fp12_one();
#pragma unroll 1
  for (uint32_t s = 0; s < CK_STEPS; ++s) {
    const bool dbl = ck_step_is_dbl(s);
    if (s != 0 && dbl) f = fp12_sqr(f);
    CkLine l;
    if (dbl) {
      ck_line_dbl(T, l);
    } else {
      const G2A qa = q();
      ck_line_add(T, qa.x, qa.y, l);
    }
    f = fp12_mul_014(f, l.c0, fp2_mul_fp(l.c1, px), fp2_mul_fp(l.c4, py));
  }
  return fp12_conj(f);
}

// ---- final exponentiation in pieces (pairing.h final_exp_cubed)
// f^-1 = (f0 t6^-1, -f1 t6^-1) with t6 = f0^2 - v f1^2 (field.h fp12_inv); t6^-1 by fp6_inv, whose one inversion
// (of the Fp2 value t) becomes an inversion of N(t) in Fp, batched across the checks
struct CkInv {
  Fp6 c;  // fp6_inv's (c0, c1, c2) of t6
  Fp2 t;  // fp6_inv's t: t6^-1 = c / t
};
DGI Fp ck_fe1(const Fp12& f, CkInv& out) {
  const Fp6 a = fp6_sub(fp6_mul(f.c0, f.c0), fp6_mul_v(fp6_mul(f.c1, f.c1)));
  out.c.c0 = fp2_sub(fp2_sqr(a.c0), fp2_mul_xi(fp2_mul(a.c1, a.c2)));
  out.c.c1 = fp2_sub(fp2_mul_xi(fp2_sqr(a.c2)), fp2_mul(a.c0, a.c1));
  out.c.c2 = fp2_sub(fp2_sqr(a.c1), fp2_mul(a.c0, a.c2));
  out.t = fp2_add(fp2_mul_xi(fp2_add(fp2_mul(a.c2, out.c.c1), fp2_mul(a.c1, out.c.c2))), fp2_mul(a.c0, out.c.c0));
  return fp2_norm(out.t);
}
// f^-1 given inv_n = 1 / N(t)
DGI Fp12 ck_inv(const Fp12& f, const CkInv& in, const Fp& inv_n) {
  const Fp2 ti{fp_mul(in.t.c0, inv_n), fp_neg(fp_mul(in.t.c1, inv_n))};  // fp2_inv(t)
  const Fp6 t6i{fp2_mul(in.c.c0, ti), fp2_mul(in.c.c1, ti), fp2_mul(in.c.c2, ti)};
  return Fp12{fp6_mul(f.c0, t6i), fp6_neg(fp6_mul(f.c1, t6i))};
}
// a * op(b), op = frob^nfrob then conj if `conj` (the products of final_exp_cubed)
DGI Fp12 ck_mul_op(const Fp12& a, Fp12 b, uint32_t nfrob, uint32_t conj) {
#pragma unroll 1
  for (uint32_t i = 0; i < nfrob; ++i) b = fp12_frob(b);
  if (conj) b = fp12_conj(b);
  return fp12_mul(a, b);
}
// the compressed chain of x^|z| (pairing.h cyc_exp_z): the six powers x^(2^k), k the set bits of |z|, and the norms
// of their denominators 4 g2; returns whether a denominator is zero (then the check takes the uncompressed chain)
template <class Put>
DGI bool ck_expsq(const Fp12& x, Put put) {
  CycC c{x.c1.c0, x.c0.c2, x.c0.c1, x.c1.c2};
  bool zero = false;
  int n = 0;
#pragma unroll 1
  for (int k = 1; k <= 63; ++k) {
    c = cyc_sqr_c(c);
    if ((Z_ABS >> k) & 1) {
      const Fp2 d = fp2_dbl(fp2_dbl(c.g2));
      zero |= fp2_is_zero(d);
      put(n++, c, fp2_norm(d));
    }
  }
  return zero;
}
// One Karabina squaring (pairing.h cyc_sqr_c) split over the two lanes of a check (k_ck_expsq2, the latency form of
// the isolation): lane half 0 owns (u, v) = (g2, g3) and has received (x, y) = (g4, g5); half 1 owns (g4, g5) and has
// received (g2, g3).  Each lane squares the received pair (three Fp2 squarings instead of six per lane) and outputs
// its own next pair: half 0 (h2, h3), half 1 (h4, h5); the lanes then swap their outputs.
DGI void ck_cyc_half(uint32_t half, const Fp2& u, const Fp2& v, const Fp2& x, const Fp2& y, Fp2& o1, Fp2& o2) {
  const Fp2 sx = DG_FP4_SQR2(x), sy = DG_FP4_SQR2(y);
  const Fp2 b = fp2_sub(fp2_sub(DG_FP4_SQR2(fp2_add(x, y)), sx), sy);  // 2 x y
  const Fp2 a = fp2_add(sx, fp2_mul_xi(sy));
  const Fp2 a3 = fp2_add(fp2_dbl(a), a);
  if (half == 0) {  // h2 = 2 g2 + 3 xi b45, h3 = 3 a45 - 2 g3
    const Fp2 t = fp2_mul_xi(b);
    o1 = fp2_add(fp2_dbl(u), fp2_add(fp2_dbl(t), t));
    o2 = fp2_sub(a3, fp2_dbl(v));
  } else {  // h4 = 3 a23 - 2 g4, h5 = 2 g5 + 3 b23
    o1 = fp2_sub(a3, fp2_dbl(u));
    o2 = fp2_add(fp2_dbl(v), fp2_add(fp2_dbl(b), b));
  }
}
// x^z from the six compressed powers and the inverses of their denominators' norms (get(i, c, nv))
template <class Get>
DGI Fp12 ck_expdec(Get get) {
  Fp12 acc = fp12_one();
#pragma unroll 1
  for (int i = CK_NPOW - 1; i >= 0; --i) {
    CycC c;
    Fp nv;
    get(i, c, nv);
    const Fp2 d = fp2_dbl(fp2_dbl(c.g2));
    const Fp2 inv{fp_mul(d.c0, nv), fp_neg(fp_mul(d.c1, nv))};  // 1 / d = conj(d) / N(d)
    acc = fp12_mul(acc, cyc_decompress(c, inv));
  }
  return fp12_conj(acc);
}
// the six norms nv(i) (none zero) replaced by their inverses (Montgomery's trick: one Fp inversion, 15 products)
template <class Ld, class St>
DGI void ck_inv6(Ld ld, St st) {
  Fp pre[CK_NPOW];
  pre[0] = ld(0);
#pragma unroll 1
  for (int i = 1; i < CK_NPOW; ++i) pre[i] = fp_mul(pre[i - 1], ld(i));
  Fp inv = fp_inv(pre[CK_NPOW - 1]);
#pragma unroll 1
  for (int i = CK_NPOW - 1; i > 0; --i) {
    const Fp n = ld(i);
    st(i, fp_mul(inv, pre[i - 1]));
    inv = fp_mul(inv, n);
  }
  st(0, inv);
}
// x^z by the uncompressed chain (pairing.h cyc_exp_z's fallback)
DGI Fp12 ck_exp_plain(const Fp12& a) {
  Fp12 acc = a;
#pragma unroll 1
  for (int b = 62; b >= 0; --b) {
    acc = fp12_cyc_sqr(acc);
    if ((Z_ABS >> b) & 1) acc = fp12_mul(acc, a);
  }
  return fp12_conj(acc);
}

// curve.h g2_in_subgroup_aff with the accumulator in LDS (g2_dbl_lds / g2_madd_lds, serialised products): the same
// test, [|z|]P by double-and-add and psi(P) == [z]P compared projectively, without a register-resident Jacobian
// point beside the formulas' temporaries (inlined as in g2_in_subgroup_aff, 221 spilled VGPRs at 2 waves per SIMD)
template <class Slot>
DGI bool ck_in_subgroup(const Fp2& x, const Fp2& y, Slot& acc) {
  acc.x = x;
  acc.y = y;
  acc.z = fp2_one();
#pragma unroll 1
  for (int b = 62; b >= 0; --b) {
    g2_dbl_lds(acc);
    if ((Z_ABS >> b) & 1) g2_madd_lds(acc, x, y);
  }
  const Fp2 az = acc.z;
  if (fp2_is_zero(az)) return false;
  const Fp2 zz = fp2_sqr_seq(az);
  const Fp2 px = fp2_mul_seq(fp2_conj(x), fp2_const(PSI_CX));
  if (!fp2_eq(fp2_mul_seq(px, zz), acc.x)) return false;
  const Fp2 py = fp2_mul_seq(fp2_conj(y), fp2_const(PSI_CY));
  return fp2_eq(fp2_mul_seq(py, fp2_mul_seq(zz, az)), fp2_neg(acc.y));
}
// ---- the G2 sum b = sum rho_i S_i of a group check off the lane's stack (DG_CK_SPLIT, default on): the four-point
// sign-aligned column form of curve.h jac_msm4_sac (the same recoding: recover.h rs_recode; the same table
// T[u] = P0 + u1 P1 + u2 P2 + u3 P3), but the 8-entry table is AFFINE, built in three levels of batched affine pair
// additions (curve.h g2_aff_kind / g2_aff_den / g2_aff_sum: chord, tangent, P + (-P), identity operands -- members
// may repeat or cancel) into an HBM table, and the column loop adds its entries with mixed additions into an LDS
// accumulator (g2_madd_lds).  Inside k_ck_prep the Jacobian table lived in scratch (6.1 KB private segment, ~54 GB
// of scratch traffic per launch at C5).  b's affine form comes from one batch inversion of N(Z) across the chunk.
// member m of a check (the identity past the live members)
DGI G2A ck_member(const CkState& c, const G2AStore* S, uint32_t m) {
  return m < c.nl ? load_g2a(S[c.live[m]]) : G2A{fp2_zero(), fp2_zero(), true};
}
// table level l, element e: the operands A (an earlier entry, or P0) and B = P[pb] of the entry dst it writes
template <class GetT>
DGI bool ck_tab_operands(uint32_t l, uint32_t e, const CkState& c, const G2AStore* S, GetT getT, G2A& A, G2A& B,
                         uint32_t& dst) {
  uint32_t src, pb;
  if (!rs_level(l, e, src, pb, dst)) return false;
  A = src ? getT(src) : ck_member(c, S, 0);
  B = ck_member(c, S, pb);
  return true;
}
// the column loop over the affine table (getT(u) = T[u]), accumulator `acc` (LDS slot on the device)
template <class GetT, class Slot>
DGI void ck_sac_g2(const RsDigits& d, GetT getT, Slot& acc) {
  acc.x = fp2_zero();
  acc.y = fp2_zero();
  acc.z = fp2_zero();
#pragma unroll 1
  for (int c = 64; c >= 0; --c) {
    if (c < 64) g2_dbl_lds(acc);
    uint32_t e;
    bool pos;
    if (c == 64) {
      e = d.top;
      pos = true;
    } else {
      e = (uint32_t)((d.um[0] >> c) & 1u) | (uint32_t)((d.um[1] >> c) & 1u) << 1 | (uint32_t)((d.um[2] >> c) & 1u) << 2;
      pos = (d.sgn >> c) & 1u;
    }
    const G2A t = getT(e);
    if (!t.inf) g2_madd_lds(acc, t.x, pos ? t.y : fp2_neg(t.y));
  }
  if (d.even) {
    const G2A t = getT(0);
    if (!t.inf) g2_madd_lds(acc, t.x, fp2_neg(t.y));
  }
}
// affine form of a Jacobian b given ninv = 1 / N(Z) (0 for the identity)
DGI G2A ck_g2_affine(const G2J& b, const Fp& ninv) {
  if (fp2_is_zero(b.z)) return G2A{fp2_zero(), fp2_zero(), true};
  const Fp2 zi = Fp2{fp_mul_seq(b.z.c0, ninv), fp_neg(fp_mul_seq(b.z.c1, ninv))};
  const Fp2 zi2 = fp2_sqr_seq(zi);
  return G2A{fp2_mul_seq(b.x, zi2), fp2_mul_seq(b.y, fp2_mul_seq(zi2, zi)), false};
}

#if defined(__HIP__)
static_assert(CK_GRP == GRP, "one group per check");
// the partner lane's value (lanes 2i, 2i + 1 swap: DPP quad_perm [1, 0, 3, 2]); both lanes must be active
__device__ __forceinline__ uint32_t ck_xpair(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xF, 0xF, false);
}
__device__ __forceinline__ Fp2 ck_xpair(const Fp2& a) {
  Fp2 r;
#pragma unroll
  for (int i = 0; i < 12; ++i) {
    r.c0.l[i] = ck_xpair(a.c0.l[i]);
    r.c1.l[i] = ck_xpair(a.c1.l[i]);
  }
  return r;
}

// H_r = h_eff(Q_r) and its 68 lines (once per Recover call and round): rl[s * R + r]; hinf[r]: H_r is the identity
// (kernels_check_a.hip)
#if DG_TU_CHECK == 1
DG_KERNEL void __launch_bounds__(64, DG_CK_WAVES) k_ck_round_lines(uint32_t R, const G2JStore* Q, CkLine* rl, uint8_t* hinf) {
  DG_HI();
  const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= R) return;
  const G2A h = g2_to_aff(g2_clear_cofactor(load_g2j(Q[r])));
  hinf[r] = h.inf ? 1 : 0;
  if (h.inf) return;
  ck_lines(h.x, h.y, [&](uint32_t s, const CkLine& l) { rl[(size_t)s * R + r] = l; });
}
// the G2 subgroup checks of the members (one lane per member slot 4 (off + g) + m of the list), ahead of k_ck_prep:
// a dense single-purpose launch instead of up to four checks in a row inside a k_ck_prep lane.  A member outside G2
// gets group_combine's decode-error verdict here (fin = FIN_DONE, so group_combine leaves it out); a recheck was
// subgroup-checked by its group.
DG_KERNEL void __launch_bounds__(64, DG_CK_SUB_WAVES) k_ck_sub(uint32_t G, uint32_t off, const uint32_t* glist,
                                                                const G2AStore* S, uint8_t* status, uint8_t* fin) {
  DG_HI();
  const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  __shared__ G2JStore s_acc[64];
  if (g >= 4 * G) return;
  const uint32_t i = glist[4 + 4 * (size_t)off + g];
  if (i == ~0u || fin[i] == FIN_RECHECK) return;
  const G2A s = load_g2a(S[i]);
  if (!s.inf && !ck_in_subgroup(s.x, s.y, s_acc[threadIdx.x])) {
    status[i] = DG_ST_SIG_DECODE_;
    fin[i] = FIN_DONE;
  }
}
// the check's members (glist group off + g), as verify_group: subgroup checks (unless k_ck_sub ran: subgroup = 0),
// the weighted sums (group_combine)
// (g2m != null: the G2 sum of a group is left to k_ck_tab_* / k_ck_sac / k_ck_bfin -- g2m[g] = 1 and dig[g] its
// column digits -- and so is np)
DGI void ck_prep(uint32_t G, uint32_t off, const uint32_t* glist, uint32_t k, const uint64_t* seedp, const G1AStore* keys,
                 const uint32_t* item_slot, const uint8_t* hinf, const G2AStore* S, uint8_t* status, uint8_t* fin,
                 uint32_t subgroup, unsigned long long* cnt, CkState* st, uint8_t* g2m, RsDigits* dig) {
  const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= G) return;
  const uint32_t* mem = glist + 4 + 4 * (size_t)(off + g);
  uint32_t n = 0;
  while (n < GRP && mem[n] != ~0u) ++n;
  atomicAdd(&cnt[n - 1], 1ull);
  G1A a{fp_zero(), fp_zero(), true};
  G2A b{fp2_zero(), fp2_zero(), true};
  CkState c;
  uint64_t rho[GRP];
  const uint32_t nl = group_combine(mem, n, *seedp, keys, item_slot, S, status, fin, subgroup, a, b, c.live, rho);
  c.round = mem[0] / k;
  c.n = n;
  c.nl = nl;
  if (nl == 0) {
    a = G1A{fp_zero(), fp_zero(), true};
    b = G2A{fp2_zero(), fp2_zero(), true};
  }
  const bool later = n > 1 && nl > 0;  // b from the table kernels
  {
    g2m[g] = later ? 1 : 0;
    if (later) {
      const uint64_t d[4] = {rho[0], rho[1], rho[2], rho[3]};
      dig[g] = rs_recode(d);
    }
  }
  c.np = ((!a.inf && !hinf[c.round]) ? 1u : 0u) | (!b.inf ? 2u : 0u);
  store_g1a(c.a, a);
  store_g2a(c.b, b);
  st[g] = c;
}
DG_KERNEL void __launch_bounds__(64, DG_CK_WAVES2) k_ck_prep(uint32_t G, uint32_t off, const uint32_t* glist, uint32_t k,
                                                  const uint64_t* seedp, const G1AStore* keys, const uint32_t* item_slot,
                                                  const uint8_t* hinf, const G2AStore* S, uint8_t* status, uint8_t* fin,
                                                  uint32_t subgroup, unsigned long long* cnt, CkState* st,
                                                  uint8_t* g2m, RsDigits* dig) {
  DG_HI();
  ck_prep(G, off, glist, k, seedp, keys, item_slot, hinf, S, status, fin, subgroup, cnt, st, g2m, dig);
}
// the lines of the pair (-g1, b): l2[s * G + g]
DG_KERNEL void __launch_bounds__(64, DG_CK_L2_WAVES) k_ck_lines2(uint32_t G, const uint32_t* gcnt, const CkState* st,
                                                                 CkLine* l2) {
  DG_HI();
  const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  if (ck_dead(g, G, gcnt) || !(st[g].np & 2)) return;
  const G2A b = load_g2a(st[g].b);
  ck_lines(b.x, b.y, [&](uint32_t s, const CkLine& l) { l2[(size_t)s * G + g] = l; });
}
// The six compressed powers of x^|z| (ck_expsq) sn[i * G + g], their denominators' norms nv[i * G + g], zero[g] (a
// lane with a zero denominator also appends itself to zl: zl[0] the count, zl[1..] the lanes; x = 1 -- the dead
// checks, whose verdict k_ck_final ignores -- skips the chain: 1^z = 1, zero[g] = 2), with two lanes per check (lanes
// 2g, 2g + 1 of a wave: ck_cyc_half, the outputs swapped by a DPP quad permutation): half the dependent products per
// squaring for the isolation's few checks, and no spills (the one-lane form spilled 79 VGPRs; C5 15.3 -> 15.6 k)
DG_KERNEL void __launch_bounds__(64, DG_CK_WAVES2) k_ck_expsq2(uint32_t G, const uint32_t* gcnt, const Fp12* X, CycC* sn,
                                                               Fp* nv, uint8_t* zero, uint32_t* zl) {
  DG_HI();
  const uint32_t lane = blockIdx.x * blockDim.x + threadIdx.x, g = lane >> 1, half = lane & 1;
  if (ck_dead(g, G, gcnt)) return;  // (both lanes of a check alike)
  const Fp12 x = X[g];
  if (fp12_is_one(x)) {
    if (!half) zero[g] = 2;
    return;
  }
  // CycC{g2, g3, g4, g5} = {x.c1.c0, x.c0.c2, x.c0.c1, x.c1.c2}
  Fp2 u = half ? x.c0.c1 : x.c1.c0, v = half ? x.c1.c2 : x.c0.c2;
  Fp2 p = half ? x.c1.c0 : x.c0.c1, q = half ? x.c0.c2 : x.c1.c2;
  bool z = false;
  int n = 0;
#pragma unroll 1
  for (int k = 1; k <= 63; ++k) {
    ck_cyc_half(half, u, v, p, q, u, v);
    p = ck_xpair(u);
    q = ck_xpair(v);
    if ((Z_ABS >> k) & 1) {
      CycC* c = sn + (size_t)n * G + g;
      if (!half) {
        c->g2 = u;
        c->g3 = v;
        const Fp2 d = fp2_dbl(fp2_dbl(u));
        z |= fp2_is_zero(d);
        nv[(size_t)n * G + g] = fp2_norm(d);
      } else {
        c->g4 = u;
        c->g5 = v;
      }
      ++n;
    }
  }
  if (!half) {
    zero[g] = z ? 1 : 0;
    if (z) zl[1 + atomicAdd(zl, 1u)] = g;
  }
}
// the verdicts of the group / single checks of Recover's pass (good[g]: the check held, k_ck_final): a passed group
// accepts its members (error probability <= 2^-63 each), a failed group sends them to their own checks (FIN_RECHECK),
// a single check is kyber's bls.Verify verdict
DG_KERNEL void __launch_bounds__(128) k_ck_verdict(uint32_t G, const CkState* st, const uint8_t* good_, uint8_t* status,
                                                   uint8_t* fin) {
  DG_HI();
  const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= G) return;
  const CkState& c = st[g];
  if (c.nl == 0) return;
  const bool good = good_[g] != 0;
  if (c.n == 1) {
    status[c.live[0]] = good ? DG_ST_OK_ : DG_ST_BAD_SIG_;
    fin[c.live[0]] = FIN_DONE;
    return;
  }
  for (uint32_t m = 0; m < c.nl; ++m) {
    if (good) status[c.live[m]] = DG_ST_OK_;
    fin[c.live[m]] = good ? FIN_DONE : FIN_RECHECK;
  }
}
#else
DG_KERNEL void __launch_bounds__(64, DG_CK_WAVES) k_ck_round_lines(uint32_t R, const G2JStore* Q, CkLine* rl, uint8_t* hinf);
DG_KERNEL void __launch_bounds__(64, DG_CK_WAVES2) k_ck_prep(uint32_t G, uint32_t off, const uint32_t* glist, uint32_t k,
                                                  const uint64_t* seedp, const G1AStore* keys, const uint32_t* item_slot,
                                                  const uint8_t* hinf, const G2AStore* S, uint8_t* status, uint8_t* fin,
                                                  uint32_t subgroup, unsigned long long* cnt, CkState* st,
                                                  uint8_t* g2m, RsDigits* dig);
DG_KERNEL void __launch_bounds__(64, DG_CK_SUB_WAVES) k_ck_sub(uint32_t G, uint32_t off, const uint32_t* glist,
                                                                const G2AStore* S, uint8_t* status, uint8_t* fin);
DG_KERNEL void __launch_bounds__(64, DG_CK_L2_WAVES) k_ck_lines2(uint32_t G, const uint32_t* gcnt, const CkState* st,
                                                                 CkLine* l2);
DG_KERNEL void __launch_bounds__(64, DG_CK_WAVES2) k_ck_expsq2(uint32_t G, const uint32_t* gcnt, const Fp12* X, CycC* sn,
                                                               Fp* nv, uint8_t* zero, uint32_t* zl);
DG_KERNEL void __launch_bounds__(128) k_ck_verdict(uint32_t G, const CkState* st, const uint8_t* good_, uint8_t* status,
                                                   uint8_t* fin);
#endif
// (kernels_check_f.hip)
#if DG_TU_CHECK == 6
// the easy part of the final exponentiation: F2[g] = f1 frob^2(f1), f1 = f^-1 conj(f); f^-1 by ck_fe1 / ck_inv with the
// one Fp inversion of the check in the lane (field.h fp_inv, safegcd) -- no batch inversion across the checks.  Lane 0
// also empties the CK_NEXP work lists of k_ck_explain (zl + z (G + 1), z < CK_NEXP).
// (two != 0: F holds the two pairs' values of xr.h k_xg_miller, F[g] and F[G + g]; f is their product)
DG_KERNEL void __launch_bounds__(64, DG_CK_WAVES) k_ck_easy(uint32_t G, const uint32_t* gcnt, uint32_t two, const Fp12* F,
                                                            Fp12* F2, uint32_t* zl) {
  DG_HI();
  const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g == 0 && G)
#pragma unroll 1
    for (uint32_t z = 0; z < CK_NEXP; ++z) zl[(size_t)z * (G + 1)] = 0;
  if (ck_dead(g, G, gcnt)) return;
  const Fp12 f = two ? fp12_mul(F[g], F[(size_t)G + g]) : F[g];
  CkInv c;
  const Fp n = ck_fe1(f, c);
  const Fp12 f1 = ck_mul_op(ck_inv(f, c, fp_inv(n)), f, 0, 1);
  F2[g] = ck_mul_op(f1, f1, 2, 0);
}
#else
DG_KERNEL void __launch_bounds__(64, DG_CK_WAVES) k_ck_easy(uint32_t G, const uint32_t* gcnt, uint32_t two, const Fp12* F,
                                                            Fp12* F2, uint32_t* zl);
#endif
// the Miller value of every check (kernels_check_b.hip): both pairs in one lane, the squarings shared
#if DG_TU_CHECK == 2
DG_KERNEL void __launch_bounds__(64, DG_CK_WAVES) k_ck_miller(uint32_t G, const uint32_t* gcnt, uint32_t R,
                                                              const CkState* st, const CkLine* rl, const CkLine* l2,
                                                              Fp12* F) {
  DG_HI();
  const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  if (ck_dead(g, G, gcnt)) return;
  const uint32_t np = st[g].np, r = st[g].round;
  const Fp ax = st[g].a.x, ay = st[g].a.y;
  const auto line = [&](uint32_t s, uint32_t pair) { return pair ? l2[(size_t)s * G + g] : rl[(size_t)s * R + r]; };
  __shared__ uint32_t s_f[144 * 64];  // the accumulators: one 576 B column per lane (fpd.h Fd12Col)
  Fd12Col<64> f{s_f + threadIdx.x};
  F[g] = ck_miller_col(np, ax, ay, line, f);
}
#else
DG_KERNEL void __launch_bounds__(64, DG_CK_WAVES) k_ck_miller(uint32_t G, const uint32_t* gcnt, uint32_t R,
                                                              const CkState* st, const CkLine* rl, const CkLine* l2,
                                                              Fp12* F);
#endif
// the end of final_exp_cubed and the check's verdict (kernels_check_c.hip): T = (a^z)^z frob^2(a) (k_ck_expdec's
// product), b = T conj(a), c = f2^3, good[g] = (no pair, or b c == 1)
#if DG_TU_CHECK == 3
DG_KERNEL void __launch_bounds__(64, DG_CK_WAVES) k_ck_final(uint32_t G, const uint32_t* gcnt, const CkState* st,
                                                             const Fp12* T, const Fp12* A, const Fp12* F2, uint8_t* good) {
  DG_HI();
  const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  if (ck_dead(g, G, gcnt)) return;
  const Fp12 c = ck_mul_op(ck_mul_op(F2[g], F2[g], 0, 0), F2[g], 0, 0);
  const Fp12 res = ck_mul_op(ck_mul_op(T[g], A[g], 0, 1), c, 0, 0);
  good[g] = st[g].np == 0 || fp12_is_one(res) ? 1 : 0;
}
#else
DG_KERNEL void __launch_bounds__(64, DG_CK_WAVES) k_ck_final(uint32_t G, const uint32_t* gcnt, const CkState* st,
                                                             const Fp12* T, const Fp12* A, const Fp12* F2, uint8_t* good);
#endif
// x^z from the compressed powers (kernels_check_d.hip): the six norms inverted in the lane (ck_inv6, in place), the
// decompressed product, then out[g] = x^z op(Y[g]) when Y is given (op: frob^nfrob, then conj if `conj` -- the hard
// part's next factor, ck_mul_op); lanes whose chain hit a zero denominator are left to k_ck_explain
#if DG_TU_CHECK == 4
DG_KERNEL void __launch_bounds__(64, DG_CK_WAVES) k_ck_expdec(uint32_t G, const uint32_t* gcnt, const CycC* sn, Fp* nv,
                                                              const uint8_t* zero, const Fp12* Y, uint32_t nfrob,
                                                              uint32_t conj, Fp12* out) {
  DG_HI();
  const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  if (ck_dead(g, G, gcnt) || zero[g] == 1) return;
  Fp12 x = fp12_one();  // x = 1 (zero[g] == 2, k_ck_expsq2)
  if (zero[g] == 0) {
    ck_inv6([&](int i) { return nv[(size_t)i * G + g]; }, [&](int i, const Fp& v) { nv[(size_t)i * G + g] = v; });
    x = ck_expdec([&](int i, CycC& c, Fp& n) {
      c = sn[(size_t)i * G + g];
      n = nv[(size_t)i * G + g];
    });
  }
  out[g] = Y ? ck_mul_op(x, Y[g], nfrob, conj) : x;
}
#else
DG_KERNEL void __launch_bounds__(64, DG_CK_WAVES) k_ck_expdec(uint32_t G, const uint32_t* gcnt, const CycC* sn, Fp* nv,
                                                              const uint8_t* zero, const Fp12* Y, uint32_t nfrob,
                                                              uint32_t conj, Fp12* out);
#endif
// x^z by the uncompressed chain for the lanes with a zero Karabina denominator (kernels_check_e.hip)
// over the work list zl (k_ck_expsq2) with a fixed grid of CK_EXPLAIN_LANES lanes striding it; every lane exits when
// the list is done
constexpr uint32_t CK_EXPLAIN_LANES = 4096;
// the split G2 sums (kernels_check_e.hip): table levels, column loop, affine form.  T4: the affine table entries
// SoA (entry u of check g at T4 + u * RC_Q * G + g, stride G), tinf[u * G + g] its identity flag.
#if DG_TU_CHECK == 5
DGI G2A ck_tab_get(const uint4* T4, const uint8_t* tinf, uint32_t G, uint32_t g, uint32_t u) {
  G2A t;
  t.inf = tinf[(size_t)u * G + g] != 0;
  rc_ld(T4 + (size_t)u * RC_Q * G + g, G, t.x, t.y);
  return t;
}
DGI void ck_tab_put(uint4* T4, uint8_t* tinf, uint32_t G, uint32_t g, uint32_t u, const G2A& t) {
  tinf[(size_t)u * G + g] = t.inf ? 1 : 0;
  rc_st(T4 + (size_t)u * RC_Q * G + g, G, t.inf ? fp2_zero() : t.x, t.inf ? fp2_zero() : t.y);
}
// lane e G + g: den[lane] = N(d) of element e of level l (1 where nothing is inverted); level 0 also stores T0 = P0
DG_KERNEL void __launch_bounds__(64, DG_CK_WAVES2) k_ck_tab_den(uint32_t l, uint32_t G, const CkState* st,
                                                               const uint8_t* g2m, const G2AStore* S, uint4* T4,
                                                               uint8_t* tinf, Fp* den) {
  DG_HI();
  const uint32_t lane = blockIdx.x * blockDim.x + threadIdx.x;
  if (lane >= 3 * G) return;
  const uint32_t g = lane % G, e = lane / G;
  Fp v = fp_one();
  G2A A, B;
  uint32_t dst;
  if (g2m[g] && ck_tab_operands(l, e, st[g], S, [&](uint32_t u) { return ck_tab_get(T4, tinf, G, g, u); }, A, B, dst)) {
    if (l == 0 && e == 0) ck_tab_put(T4, tinf, G, g, 0, ck_member(st[g], S, 0));
    v = g2_aff_den(A, B, g2_aff_kind(A, B));
  }
  den[lane] = v;
}
DG_KERNEL void __launch_bounds__(64, DG_CK_WAVES2) k_ck_tab_add(uint32_t l, uint32_t G, const CkState* st,
                                                               const uint8_t* g2m, const G2AStore* S, uint4* T4,
                                                               uint8_t* tinf, const Fp* dinv) {
  DG_HI();
  const uint32_t lane = blockIdx.x * blockDim.x + threadIdx.x;
  if (lane >= 3 * G) return;
  const uint32_t g = lane % G, e = lane / G;
  G2A A, B;
  uint32_t dst;
  if (!g2m[g] || !ck_tab_operands(l, e, st[g], S, [&](uint32_t u) { return ck_tab_get(T4, tinf, G, g, u); }, A, B, dst))
    return;
  ck_tab_put(T4, tinf, G, g, dst, g2_aff_sum(A, B, g2_aff_kind(A, B), dinv[lane]));
}
// the column loop: bj[g] = b (Jacobian), bn[g] = N(Z) (1 for the lanes not on this path)
DG_KERNEL void __launch_bounds__(64, DG_CK_WAVES2) k_ck_sac(uint32_t G, const uint8_t* g2m, const RsDigits* dig,
                                                           const uint4* T4, const uint8_t* tinf, G2JStore* bj, Fp* bn) {
  DG_HI();
  const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  __shared__ G2JStore s_acc[64];
  if (g >= G) return;
  if (!g2m[g]) {
    bn[g] = fp_one();
    return;
  }
  G2JStore& acc = s_acc[threadIdx.x];
  ck_sac_g2(dig[g], [&](uint32_t u) { return ck_tab_get(T4, tinf, G, g, u); }, acc);
  bj[g] = acc;
  bn[g] = fp2_norm(acc.z);
}
// st[g].b = the affine b, and np
DG_KERNEL void __launch_bounds__(64, DG_CK_WAVES2) k_ck_bfin(uint32_t G, const uint8_t* g2m, const G2JStore* bj,
                                                            const Fp* bni, const uint8_t* hinf, CkState* st) {
  DG_HI();
  const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= G || !g2m[g]) return;
  const G2A b = ck_g2_affine(load_g2j(bj[g]), bni[g]);
  store_g2a(st[g].b, b);
  const G1A a = load_g1a(st[g].a);
  st[g].np = ((!a.inf && !hinf[st[g].round]) ? 1u : 0u) | (!b.inf ? 2u : 0u);
}
DG_KERNEL void __launch_bounds__(64, DG_CK_WAVES) k_ck_explain(const uint32_t* zl, const Fp12* X, const Fp12* Y,
                                                               uint32_t nfrob, uint32_t conj, Fp12* out) {
  DG_HI();
  const uint32_t n = zl[0];
  for (uint32_t j = blockIdx.x * blockDim.x + threadIdx.x; j < n; j += gridDim.x * blockDim.x) {
    const uint32_t g = zl[1 + j];
    const Fp12 x = ck_exp_plain(X[g]);
    out[g] = Y ? ck_mul_op(x, Y[g], nfrob, conj) : x;
  }
}
#else
DG_KERNEL void __launch_bounds__(64, DG_CK_WAVES2) k_ck_tab_den(uint32_t l, uint32_t G, const CkState* st,
                                                               const uint8_t* g2m, const G2AStore* S, uint4* T4,
                                                               uint8_t* tinf, Fp* den);
DG_KERNEL void __launch_bounds__(64, DG_CK_WAVES2) k_ck_tab_add(uint32_t l, uint32_t G, const CkState* st,
                                                               const uint8_t* g2m, const G2AStore* S, uint4* T4,
                                                               uint8_t* tinf, const Fp* dinv);
DG_KERNEL void __launch_bounds__(64, DG_CK_WAVES2) k_ck_sac(uint32_t G, const uint8_t* g2m, const RsDigits* dig,
                                                           const uint4* T4, const uint8_t* tinf, G2JStore* bj, Fp* bn);
DG_KERNEL void __launch_bounds__(64, DG_CK_WAVES2) k_ck_bfin(uint32_t G, const uint8_t* g2m, const G2JStore* bj,
                                                            const Fp* bni, const uint8_t* hinf, CkState* st);
DG_KERNEL void __launch_bounds__(64, DG_CK_WAVES) k_ck_explain(const uint32_t* zl, const Fp12* X, const Fp12* Y,
                                                               uint32_t nfrob, uint32_t conj, Fp12* out);
#endif
#endif

}  // namespace dg
