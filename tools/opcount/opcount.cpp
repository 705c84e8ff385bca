// Instrumented HOST build of the kernels' device arithmetic (drand_amd/csrc/*.h compiled with g++ and
// -DDG_OPCOUNT): counts the Montgomery multiplications and squarings each kernel's per-unit body
// executes, so bench.py can turn kernel time into algorithmic multiply-adds/s.
// Tooling only -- never linked into the product library.
#include <string.h>

#include <vector>

#include "../../drand_amd/csrc/kernels.h"

namespace dg {
thread_local uint64_t g_fp_mul_count = 0, g_fp_sqr_count = 0, g_fp_inv_count = 0;
}
using namespace dg;

static void reset() { g_fp_mul_count = g_fp_sqr_count = g_fp_inv_count = 0; }
static void take(uint64_t* out) {
  out[0] = g_fp_mul_count;
  out[1] = g_fp_sqr_count;
  out[2] = g_fp_inv_count;
}

extern "C" {
// out[0..1] = (mul, sqr) of hash_to_g2_uncleared(msg) -- k_h2c_uncleared per round
void oc_h2c_uncleared(const uint8_t* msg, uint32_t len, const uint8_t* dst, uint32_t dl, uint64_t* out) {
  // as k_h2c_uncleared computes one round (word-wise expand_message_xmd for 32 B messages; the two-lane
  // kernel repeats the final addition and normalisation in both lanes: not counted, the algorithm needs one)
  static XmdTail T;
  xmd_tail_build(T, dst, dl);
  reset();
  Fp2 u[2];
  if (len == 32)
    hash_to_field_xmd32(u, msg, &T);
  else
    hash_to_field_fp2x2(u, msg, len, dst, dl);
  G2J q[2];
  for (int h = 0; h < 2; ++h) {
    Fp2 x, y;
    sswu_g2(x, y, u[h], fp_zero(), false);
    q[h] = iso_map_g2(x, y);
  }
  G2J r = jac_from_aff(g2_to_aff(jac_add(q[0], q[1])));
  (void)r;
  take(out);
}
// the phase kernels of phases.h for one round (k_h2c_p1 / p4 per round, p2 / p3 per map item, k_exp_pm3d4
// per exponentiation): out[6 * phase + 0..2] = (mul, sqr, inv) of phase p1, exp, p2, p3, p4 (exp: one of the
// four), summed over the round's map items
void oc_h2c_phases(const uint8_t* msg, const uint8_t* dst, uint32_t dl, uint64_t* out) {
  static XmdTail T;
  xmd_tail_build(T, dst, dl);
  Fp2 u[2];
  H2cMap st[2];
  Fp e[2];
  reset();
  hash_to_field_xmd32(u, msg, &T);
  Fp nD;
  h2c_p1a(u, st, nD);
  uint64_t part[3];
  take(part);
  Fp inv_nD = fp_inv(nD);  // the batch inversion's share (3 products per value) is not counted here
  reset();
  h2c_p1b(st, inv_nD, e);
  take(out);
  for (int k = 0; k < 3; ++k) out[k] += part[k];
  G2J q[2];
  uint64_t tmp[3];
  for (int k = 3; k < 15; ++k) out[k] = 0;
  for (int h = 0; h < 2; ++h) {
    reset();
    Fp t = fp_pow_pm3d4_sos(e[h]);
    take(tmp);
    for (int k = 0; k < 3; ++k) out[3 + k] = tmp[k];
    Fp c;
    reset();
    h2c_p2(st[h], e[h], t, c);
    take(tmp);
    for (int k = 0; k < 3; ++k) out[6 + k] += tmp[k];
    Fp t2 = fp_pow_pm3d4_sos(c);
    reset();
    q[h] = h2c_p3(st[h], c, t2);
    take(tmp);
    for (int k = 0; k < 3; ++k) out[9 + k] += tmp[k];
  }
  reset();
  G2J r = jac_add(q[0], q[1]);
  Fp nZ = fp2_norm(r.z);
  take(part);
  Fp inv_nZ = fp_inv(nZ);  // from the batch inversion, not counted
  reset();
  Fp2 zinv{fp_mul(r.z.c0, inv_nZ), fp_neg(fp_mul(r.z.c1, inv_nZ))};  // as k_h2c_p4b
  G2J a = jac_from_aff(jac_to_aff_with_inv(r, zinv));
  (void)a;
  take(out + 12);
  for (int k = 0; k < 3; ++k) out[12 + k] += part[k];
}
// the decompression phases for one item: out = p1, exp, p2, p3 (mul, sqr, inv) each
int oc_dec_phases(const uint8_t* sig96, uint64_t* out) {
  DecState ds;
  Fp e, c = fp_zero();
  G2A a;
  reset();
  bool ok = dec_p1(sig96, ds, e) == 0;
  take(out);
  reset();
  Fp t = fp_pow_pm3d4_sos(e);
  take(out + 3);
  reset();
  ok = ok && dec_p2(ds, e, t, c);
  take(out + 6);
  Fp t2 = fp_pow_pm3d4_sos(c);
  reset();
  ok = ok && dec_p3(ds, c, t2, false, a);
  take(out + 9);
  return ok;
}
// g2_decompress (+ subgroup check when `subgroup`: multi-key batches; the beacon path batches it on the
// MSM window sums) -- k_decode_items per item; returns decode ok
int oc_decode_g2(const uint8_t* sig96, int subgroup, uint64_t* out) {
  reset();
  G2A a;
  bool ok = g2_decompress(a, sig96, subgroup != 0);
  take(out);
  return ok;
}
// k_round_combine per round (k = 1): W = alpha sigma, A = alpha Q (Q = uncleared hash of msg)
void oc_round_combine(const uint8_t* msg, uint32_t len, const uint8_t* dst, uint32_t dl, const uint8_t* sig96,
                      uint64_t alpha, uint64_t* out) {
  G2J q = jac_from_aff(g2_to_aff(hash_to_g2_uncleared(msg, len, dst, dl)));
  G2A s;
  g2_decompress(s, sig96, true);
  reset();
  G2J w = jac_mul_u64(jac_from_aff(s), alpha);
  G2J a = jac_mul_u64(q, alpha);
  (void)w;
  (void)a;
  take(out);
}
// one Jacobian G2 addition of two generic points (k_sum_rows / k_key_accum per point)
void oc_g2_add(const uint8_t* sig_a, const uint8_t* sig_b, uint64_t* out) {
  G2A a, b;
  g2_decompress(a, sig_a, false);
  g2_decompress(b, sig_b, false);
  G2J ja = jac_dbl(jac_from_aff(a)), jb = jac_dbl(jac_from_aff(b));  // generic Z != 1
  reset();
  G2J c = jac_add(ja, jb);
  (void)c;
  take(out);
}
// one mixed addition (Jacobian + affine): k_msm_chunks per decoded signature
void oc_g2_add_aff(const uint8_t* sig_a, const uint8_t* sig_b, uint64_t* out) {
  G2A a, b;
  g2_decompress(a, sig_a, false);
  g2_decompress(b, sig_b, false);
  G2J ja = jac_dbl(jac_from_aff(a));
  reset();
  G2J c = jac_add_aff(ja, b.x, b.y);
  (void)c;
  take(out);
}
// k_pair_miller (key pair) + k_final_check for a batch of one key
void oc_batch_final(const uint8_t* pk48, const uint8_t* sig_a, const uint8_t* sig_b, uint64_t* out) {
  G1A pk;
  g1_decompress(pk, pk48, false);
  G2A a, b;
  g2_decompress(a, sig_a, false);
  g2_decompress(b, sig_b, false);
  G2J K = jac_dbl(jac_from_aff(a)), T = jac_dbl(jac_from_aff(b));
  reset();
  G1A P[1] = {pk};
  G2A Q[1] = {g2_to_aff(g2_clear_cofactor(K))};
  Fp12 f0 = miller_loop<1>(P, Q, 1);
  P[0] = G1A{fp_const(G1_GEN_X), fp_const(G1_GEN_NEG_Y), false};
  Q[0] = g2_to_aff(T);
  Fp12 f1 = miller_loop<1>(P, Q, 1);
  bool ok = fp12_is_one(final_exp_cubed(fp12_mul(f0, f1)));
  (void)ok;
  take(out);
}
// k_verify_items per item (individual check) given uncleared hash msg and sigma
void oc_verify_item(const uint8_t* pk48, const uint8_t* msg, uint32_t len, const uint8_t* dst, uint32_t dl,
                    const uint8_t* sig96, uint64_t* out) {
  G1A pk;
  g1_decompress(pk, pk48, false);
  G2J q = hash_to_g2_uncleared(msg, len, dst, dl);
  G2A s;
  g2_decompress(s, sig96, false);
  reset();
  G2A h = g2_to_aff(g2_clear_cofactor(q));
  G1A P[2] = {pk, G1A{fp_const(G1_GEN_X), fp_const(G1_GEN_NEG_Y), false}};
  G2A Q[2] = {h, s};
  bool ok = fp12_is_one(final_exp_cubed(miller_loop<2>(P, Q, 2)));
  (void)ok;
  take(out);
}
// k_scale_items per item with nslots > 1: beta * sigma
void oc_scale_item(const uint8_t* sig96, uint64_t beta, uint64_t* out) {
  G2A s;
  g2_decompress(s, sig96, false);
  reset();
  G2J u = jac_mul_u64(jac_from_aff(s), beta);
  (void)u;
  take(out);
}
// k_recover_terms per (round, share): lambda_m * S (lambda = 32 B little-endian limbs)
void oc_recover_term(const uint8_t* sig96, const uint32_t* lam8, uint64_t* out) {
  G2A s;
  g2_decompress(s, sig96, false);
  reset();
  G2J u = g2_mul_u256_psi(s, lam8);
  (void)u;
  take(out);
}
}

// Recover's per-item pass (kernels.h k_verify_groups) for a check of m shares of one round (pk48s: m keys,
// sigs: m signatures, h from msg): m subgroup checks, for m > 1 the two weighted sums (jac_msm4_sac in G1
// and G2) and their affine forms, then one two-pair pairing check.  The cleared hash H_r is per round
// (k_clear_rounds), not counted.
extern "C" void oc_verify_group(const uint8_t* pk48s, const uint8_t* msg, const uint8_t* dst, uint32_t dl,
                                const uint8_t* sigs96, uint32_t m, uint64_t* out) {
  G2J q = hash_to_g2_uncleared(msg, 32, dst, dl);
  G2A h = g2_to_aff(g2_clear_cofactor(q));
  G1A pk[4];
  G2A s[4];
  for (uint32_t i = 0; i < m; ++i) {
    g1_decompress(pk[i], pk48s + 48 * i, false);
    g2_decompress(s[i], sigs96 + 96 * i, false);
  }
  reset();
  for (uint32_t i = 0; i < m; ++i) (void)g2_in_subgroup_aff(s[i].x, s[i].y);
  G1A a = pk[0];
  G2A b = s[0];
  if (m > 1) {
    G1J xp[4];
    G2J sp[4];
    uint64_t rho[4];
    for (uint32_t i = 0; i < 4; ++i) {
      xp[i] = i < m ? jac_from_aff(pk[i]) : jac_infinity<Fp>();
      sp[i] = i < m ? jac_from_aff(s[i]) : jac_infinity<Fp2>();
      rho[i] = i < m ? rlc_coeff(0x5eed, i) : 0;
    }
    a = g1_to_aff(jac_msm4_sac(xp, rho));
    b = g2_to_aff(jac_msm4_sac(sp, rho));
  }
  G1A P[2] = {a, G1A{fp_const(G1_GEN_X), fp_const(G1_GEN_NEG_Y), false}};
  G2A Q[2] = {h, b};
  bool ok = fp12_is_one(final_exp_cubed(miller_loop<2>(P, Q, 2)));
  (void)ok;
  take(out);
}

// Recover's per-round MSM (recover.h) for one round of t shares with index set idx: out[0..2] the odd-multiple
// tables (per share 1 tangent + 7 chord affine additions; the batch inversion's share counted as its 3 products
// per value, the inversion itself not), out[3..5] the four Straus components (k_rc_straus), out[6..8] the psi
// combination (k_rc_combine).
extern "C" void oc_recover_msm(const uint8_t* sigs96, const uint32_t* idx, uint32_t t, uint64_t* out) {
  std::vector<Fr> lam(t), pre(t);
  rc_lambdas(idx, t, lam.data(), pre.data());
  std::vector<G2A> P(t), T((size_t)t * RC_TAB);
  for (uint32_t j = 0; j < t; ++j) g2_decompress(P[j], sigs96 + 96 * j, false);
  reset();
  for (uint32_t j = 0; j < t; ++j) {
    Fp n = g2_aff_den(P[j], P[j], 2);
    g_fp_mul_count += 3;
    const G2A d = g2_aff_sum(P[j], P[j], 2, n);  // (the value of nv does not change the count)
    T[(size_t)j * RC_TAB] = P[j];
    for (uint32_t e = 1; e < RC_TAB; ++e) {
      const G2A& a = T[(size_t)j * RC_TAB + e - 1];
      n = g2_aff_den(a, d, 1);
      g_fp_mul_count += 3;
      T[(size_t)j * RC_TAB + e] = g2_aff_sum(a, d, 1, n);
    }
  }
  take(out);
  std::vector<int8_t> naf((size_t)4 * t * RC_NAF);
  for (uint32_t j = 0; j < t; ++j) {
    Fr l = lam[j];
    const bool neg = rc_signed(l);
    uint64_t d[4];
    rc_psi_digits(l, d);
    for (int i = 0; i < 4; ++i) {
      int8_t* z = naf.data() + ((size_t)i * t + j) * RC_NAF;
      rc_wnaf(d[i], z);
      if (neg)
        for (uint32_t b = 0; b < RC_NAF; ++b) z[b] = (int8_t)-z[b];
    }
  }
  std::vector<uint32_t> ev((size_t)t * RC_EV_PER_SHARE);
  G2J A[4];
  reset();
  for (int i = 0; i < 4; ++i) {
    uint32_t tail;
    const uint32_t n = rc_schedule_naf(naf.data() + (size_t)i * t * RC_NAF, t, ev.data(), tail);
    G2JStore acc{fp2_zero(), fp2_zero(), fp2_zero()};
    for (uint32_t q = 0; q < n; ++q) {
      const uint32_t v = ev[q];
      for (uint32_t d = rc_ev_dbl(v); d > 0; --d) g2_dbl_lds(acc);
      const G2A& e = T[(size_t)rc_ev_j(v) * RC_TAB + rc_ev_e(v)];
      g2_madd_lds(acc, e.x, rc_ev_neg(v) ? fp2_neg(e.y) : e.y);
    }
    for (uint32_t d = tail; d > 0; --d) g2_dbl_lds(acc);
    A[i] = G2J{acc.x, acc.y, acc.z};
  }
  take(out + 3);
  reset();
  (void)rc_combine(A[0], A[1], A[2], A[3]);
  take(out + 6);
}

// Recover's divergent-round form (recover.h k_rs_*) for one round of t shares: out[0..2] the tables (three affine
// levels, 7 additions per share with the batch inversion's 3 products per value, the psi images), out[3..5] the
// column loops of the ceil(t / RS_G) lanes and their even-digit corrections (k_rs_sac), out[6..8] the group sums.
extern "C" void oc_recover_sac(const uint8_t* sigs96, const uint32_t* idx, uint32_t t, uint64_t* out) {
  std::vector<G2A> P(t), T((size_t)t * 8);
  std::vector<RsDigits> dig(t);
  for (uint32_t j = 0; j < t; ++j) {
    g2_decompress(P[j], sigs96 + 96 * j, false);
    uint64_t d[4];
    rc_psi_digits(lagrange_at_zero(idx, t, j), d);
    dig[j] = rs_recode(d);
  }
  reset();
  for (uint32_t j = 0; j < t; ++j) {
    for (uint32_t l = 0; l < 3; ++l)
      for (uint32_t e = 0; e < 3; ++e) {
        uint32_t src, pb, dst;
        if (!rs_level(l, e, src, pb, dst)) continue;
        Fp2 px[4], py[4];
        rs_points(P[j], px, py);  // each den and add lane recomputes the psi images
        rs_points(P[j], px, py);
        const G2A a = src ? T[(size_t)j * 8 + src] : G2A{px[0], py[0], false}, b{px[pb], py[pb], false};
        const Fp n = g2_aff_den(a, b, 1);
        g_fp_mul_count += 3;
        T[(size_t)j * 8 + dst] = g2_aff_sum(a, b, 1, n);
      }
    T[(size_t)j * 8] = P[j];
  }
  take(out);
  reset();
  std::vector<G2J> part;
  for (uint32_t j0 = 0; j0 < t; j0 += RS_G) {
    const uint32_t j1 = j0 + RS_G < t ? j0 + RS_G : t;
    G2JStore acc{fp2_zero(), fp2_zero(), fp2_zero()};
    for (int c = 64; c >= 0; --c) {
      if (c < 64) g2_dbl_lds(acc);
      for (uint32_t j = j0; j < j1; ++j) {
        const RsDigits& d = dig[j];
        const uint32_t e = c == 64 ? d.top
                                   : (uint32_t)((d.um[0] >> c) & 1u) | (uint32_t)((d.um[1] >> c) & 1u) << 1 |
                                         (uint32_t)((d.um[2] >> c) & 1u) << 2;
        const G2A& x = T[(size_t)j * 8 + e];
        g2_madd_lds(acc, x.x, (c == 64 || ((d.sgn >> c) & 1u)) ? x.y : fp2_neg(x.y));
      }
    }
    for (uint32_t j = j0; j < j1; ++j)
      if (dig[j].even) g2_madd_lds(acc, T[(size_t)j * 8].x, fp2_neg(T[(size_t)j * 8].y));
    part.push_back(G2J{acc.x, acc.y, acc.z});
  }
  take(out + 3);
  reset();
  G2J s = part[0];
  for (size_t q = 1; q < part.size(); ++q) s = jac_add(s, part[q]);
  take(out + 6);
}

// The pairing-check pipeline (checks.h) for one check of m shares of one round: per kernel, in the order of out (3
// counters each): 0 k_ck_prep (m subgroup checks, the weighted sums and their affine forms), 1 k_ck_lines2 (the 68 lines
// of the pair (-g1, b)), 2 k_ck_miller, 3 k_ck_easy (f^-1 with the lane's Fp inversion, f1, f2), 4 k_ck_expsq (all
// five), 5 k_ck_expdec (all five: the lane's Montgomery trick over the 6 norms and its Fp inversion, decompression,
// the fused next factor), 6 k_ck_final, 7 k_ck_round_lines (per ROUND: h_eff and the 68 lines of H_r; the cross-round
// isolation's k_xg_hlines is the same per check).  No zero Karabina denominator occurs on these inputs (k_ck_explain:
// none).
extern "C" void oc_check_pipeline(const uint8_t* pk48s, const uint8_t* msg, const uint8_t* dst, uint32_t dl,
                                  const uint8_t* sigs96, uint32_t m, uint64_t* out) {
  G2J q = hash_to_g2_uncleared(msg, 32, dst, dl);
  G1A pk[4];
  G2A s[4];
  for (uint32_t i = 0; i < m; ++i) {
    g1_decompress(pk[i], pk48s + 48 * i, false);
    g2_decompress(s[i], sigs96 + 96 * i, false);
  }
  reset();
  const G2A h = g2_to_aff(g2_clear_cofactor(q));
  std::vector<CkLine> l1(CK_STEPS), l2(CK_STEPS);
  ck_lines(h.x, h.y, [&](uint32_t st, const CkLine& l) { l1[st] = l; });
  take(out + 21);
  reset();
  for (uint32_t i = 0; i < m; ++i) (void)g2_in_subgroup_aff(s[i].x, s[i].y);
  G1A a = pk[0];
  G2A b = s[0];
  if (m > 1) {
    G1J xp[4];
    G2J sp[4];
    uint64_t rho[4];
    for (uint32_t i = 0; i < 4; ++i) {
      xp[i] = i < m ? jac_from_aff(pk[i]) : jac_infinity<Fp>();
      sp[i] = i < m ? jac_from_aff(s[i]) : jac_infinity<Fp2>();
      rho[i] = i < m ? rlc_coeff(0x5eed, i) : 0;
    }
    a = g1_to_aff(jac_msm4_sac(xp, rho));
    b = g2_to_aff(jac_msm4_sac(sp, rho));
  }
  take(out + 0);
  reset();
  ck_lines(b.x, b.y, [&](uint32_t st, const CkLine& l) { l2[st] = l; });
  take(out + 3);
  reset();
  const Fp12 f = ck_miller(3u, a.x, a.y, [&](uint32_t st, uint32_t pair) { return pair ? l2[st] : l1[st]; });
  take(out + 6);
  reset();
  CkInv inv;
  const Fp nt = ck_fe1(f, inv);
  const Fp12 f1 = ck_mul_op(ck_inv(f, inv, fp_inv(nt)), f, 0, 1);
  const Fp12 f2 = ck_mul_op(f1, f1, 2, 0);
  take(out + 9);
  uint64_t sq[3] = {0, 0, 0}, dec[3] = {0, 0, 0};
  auto expz = [&](const Fp12& x, const Fp12* y, uint32_t nf, uint32_t cj) {
    CycC sn[CK_NPOW];
    Fp nv[CK_NPOW];
    uint64_t t[3];
    reset();
    (void)ck_expsq(x, [&](int i, const CycC& c, const Fp& n) { sn[i] = c; nv[i] = n; });
    take(t);
    for (int k = 0; k < 3; ++k) sq[k] += t[k];
    reset();
    ck_inv6([&](int i) { return nv[i]; }, [&](int i, const Fp& v) { nv[i] = v; });
    Fp12 r = ck_expdec([&](int i, CycC& c, Fp& n) { c = sn[i]; n = nv[i]; });
    if (y) r = ck_mul_op(r, *y, nf, cj);
    take(t);
    for (int k = 0; k < 3; ++k) dec[k] += t[k];
    return r;
  };
  const Fp12 t0 = expz(f2, &f2, 0, 1);
  const Fp12 t1 = expz(t0, &t0, 0, 1);
  const Fp12 aa = expz(t1, &t1, 1, 0);
  const Fp12 tt = expz(expz(aa, nullptr, 0, 0), &aa, 2, 0);
  reset();
  const Fp12 cc = ck_mul_op(ck_mul_op(f2, f2, 0, 0), f2, 0, 0);
  (void)ck_mul_op(ck_mul_op(tt, aa, 0, 1), cc, 0, 0);
  take(out + 18);
  for (int k = 0; k < 3; ++k) {
    out[12 + k] = sq[k];
    out[15 + k] = dec[k];
  }
}

// The cross-round isolation (xr.h) per unit: out[0..2] k_xq_sum (one quad side: four signatures with the coefficients
// rho), out[3..5] k_xg_prep of a level-1 group of qpg quads (2 (qpg - 1) Jacobian additions, the affine sigma sum),
// out[6..8] k_xg_prep of a level-2 quad (the affine sigma sum)
extern "C" void oc_xr_units(const uint8_t* sigs96, uint32_t qpg, uint64_t* out) {
  G2A P[4];
  for (int i = 0; i < 4; ++i) g2_decompress(P[i], sigs96 + 96 * i, false);
  uint64_t rho[4];
  for (int i = 0; i < 4; ++i) rho[i] = rlc_coeff(0x5eed, (uint64_t)i);
  G2A T[8];
  G2J acc;
  reset();
  xq_sum4([&](uint32_t m) { return P[m]; }, rho, [&](uint32_t u) { return T[u]; },
          [&](uint32_t u, const G2A& t) { T[u] = t; }, acc);
  take(out);
  // qpg distinct quad sums (other coefficients), uncounted
  std::vector<G2J> qs;
  for (uint32_t q = 0; q < qpg; ++q) {
    for (int i = 0; i < 4; ++i) rho[i] = rlc_coeff(0x5eed + q, (uint64_t)i);
    G2J a2;
    xq_sum4([&](uint32_t m) { return P[m]; }, rho, [&](uint32_t u) { return T[u]; },
            [&](uint32_t u, const G2A& t) { T[u] = t; }, a2);
    qs.push_back(a2);
  }
  reset();
  G2J h = qs[0], sg = qs[0];
  for (uint32_t q = 1; q < qpg; ++q) {
    h = jac_add(h, qs[q]);
    sg = jac_add(sg, qs[q]);
  }
  (void)g2_to_aff(sg);
  take(out + 3);
  reset();
  (void)g2_to_aff(acc);
  take(out + 6);
}
