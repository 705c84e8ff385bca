// Host build of the HIP kernels' device arithmetic (drand_amd/csrc/*.h) for step-by-step debugging
// against oracle/ on CPU.  TEST TOOL ONLY: never linked into the product library.
#include <string.h>

#include <vector>

#include <stdio.h>
#define DG_FD_CHECK 1  // fpd.h: assert the digit-form bounds in every host product, subtraction and reduction
#include "../../drand_amd/csrc/kernels.h"
static bool g_fd_bad = false;
namespace dg {
void fd_check_fail(const char* what) {
  if (!g_fd_bad) fprintf(stderr, "fpd bound violated: %s\n", what);
  g_fd_bad = true;
}
}  // namespace dg
using namespace dg;
extern "C" {
void hc_fp_mul(const uint8_t* a48, const uint8_t* b48, uint8_t* out48) {
  Fp a, b;
  fp_from_be48_plain(a, a48);
  fp_from_be48_plain(b, b48);
  fp_to_be48(out48, fp_mul(fp_to_mont(a), fp_to_mont(b)));
}
int hc_fp2_sqrt(const uint8_t* a96, uint8_t* out96) {
  Fp a0, a1;
  fp_from_be48_plain(a0, a96);
  fp_from_be48_plain(a1, a96 + 48);
  Fp2 a{fp_to_mont(a0), fp_to_mont(a1)}, r;
  bool ok = fp2_sqrt(r, a);
  fp_to_be48(out96, r.c0);
  fp_to_be48(out96 + 48, r.c1);
  return ok;
}
void hc_hash_to_g2(const uint8_t* msg, uint32_t n, const uint8_t* dst, uint32_t dl, uint8_t* out96) {
  g2_compress_aff(out96, g2_to_aff(hash_to_g2(msg, n, dst, dl)));
}
int hc_g2_roundtrip(const uint8_t* in96, uint8_t* out96) {
  G2A a;
  if (!g2_decompress(a, in96, true)) return 0;
  g2_compress_aff(out96, a);
  return 1;
}
int hc_g1_roundtrip(const uint8_t* in48, uint8_t* out48) {
  G1A a;
  if (!g1_decompress(a, in48, true)) return 0;
  g1_compress_aff(out48, a);
  return 1;
}
static const uint8_t DSTN[] = "BLS_SIG_BLS12381G2_XMD:SHA-256_SSWU_RO_NUL_";
int hc_verify(const uint8_t* pk48, const uint8_t* msg, uint32_t n, const uint8_t* sig96) {
  G1A pk;
  if (!g1_decompress(pk, pk48, true)) return 4;
  G2A s;
  if (!g2_decompress(s, sig96, true)) return 2;
  G2A h = g2_to_aff(hash_to_g2(msg, n, DSTN, 43));
  G1A P[2];
  G2A Q[2];
  int np = 0;
  if (!pk.inf && !h.inf) { P[np] = pk; Q[np] = h; ++np; }
  if (!s.inf) { P[np] = G1A{fp_const(G1_GEN_X), fp_const(G1_GEN_NEG_Y), false}; Q[np] = s; ++np; }
  if (np == 0) return 0;
  Fp12 f = miller_loop<2>(P, Q, np);
  return fp12_is_one(final_exp_cubed(f)) ? 0 : 1;
}
}
extern "C" int hc_pairing_cubed(const uint8_t* g1_48, const uint8_t* g2_96, uint8_t* out576, int variant) {
  G1A p;
  G2A q;
  if (!g1_decompress(p, g1_48, true)) return 4;
  if (!g2_decompress(q, g2_96, true)) return 2;
  Fp12 f = miller_loop<1>(&p, &q, 1);
  Fp12 r = variant == 1 ? f : final_exp_cubed(f);
  const Fp2* s[6] = {&r.c0.c0, &r.c0.c1, &r.c0.c2, &r.c1.c0, &r.c1.c1, &r.c1.c2};
  for (int i = 0; i < 6; ++i) { fp_to_be48(out576 + 96 * i, s[i]->c0); fp_to_be48(out576 + 96 * i + 48, s[i]->c1); }
  return 0;
}
extern "C" void hc_fp12_test(const uint8_t* a576, const uint8_t* b576, uint8_t* out576, int op) {
  Fp12 a, b;
  Fp2* sa[6] = {&a.c0.c0, &a.c0.c1, &a.c0.c2, &a.c1.c0, &a.c1.c1, &a.c1.c2};
  Fp2* sb[6] = {&b.c0.c0, &b.c0.c1, &b.c0.c2, &b.c1.c0, &b.c1.c1, &b.c1.c2};
  for (int i = 0; i < 6; ++i) {
    Fp x;
    fp_from_be48_plain(x, a576 + 96 * i); sa[i]->c0 = fp_to_mont(x);
    fp_from_be48_plain(x, a576 + 96 * i + 48); sa[i]->c1 = fp_to_mont(x);
    fp_from_be48_plain(x, b576 + 96 * i); sb[i]->c0 = fp_to_mont(x);
    fp_from_be48_plain(x, b576 + 96 * i + 48); sb[i]->c1 = fp_to_mont(x);
  }
  Fp12 r = op == 0 ? fp12_mul(a, b) : op == 1 ? fp12_sqr(a) : op == 2 ? fp12_inv(a) : op == 3 ? fp12_frob(a)
         : fp12_mul_014(a, b.c0.c0, b.c0.c1, b.c1.c1);
  const Fp2* s[6] = {&r.c0.c0, &r.c0.c1, &r.c0.c2, &r.c1.c0, &r.c1.c1, &r.c1.c2};
  for (int i = 0; i < 6; ++i) { fp_to_be48(out576 + 96 * i, s[i]->c0); fp_to_be48(out576 + 96 * i + 48, s[i]->c1); }
}
extern "C" int hc_verify_dbg(const uint8_t* pk48, const uint8_t* msg, uint32_t n, const uint8_t* sig96, uint8_t* h96) {
  G1A pk;
  g1_decompress(pk, pk48, true);
  G2A s;
  g2_decompress(s, sig96, true);
  G2A h = g2_to_aff(hash_to_g2(msg, n, DSTN, 43));
  g2_compress_aff(h96, h);
  G1A P[2] = {pk, G1A{fp_const(G1_GEN_X), fp_const(G1_GEN_NEG_Y), false}};
  G2A Q[2] = {h, s};
  Fp12 f1 = final_exp_cubed(miller_loop<1>(&P[0], &Q[0], 1));
  Fp12 f2 = final_exp_cubed(miller_loop<1>(&P[1], &Q[1], 1));
  Fp12 f12 = final_exp_cubed(miller_loop<2>(P, Q, 2));
  return (fp12_is_one(fp12_mul(f1, f2)) ? 1 : 0) | (fp12_is_one(f12) ? 2 : 0);
}
// safegcd inversion (fp_inv) and the Fermat cross-check, on a plain 48 B big-endian value < p
extern "C" void hc_fp_inv(const uint8_t* a48, uint8_t* out_sg48, uint8_t* out_fermat48) {
  Fp a;
  fp_from_be48_plain(a, a48);
  Fp m = fp_to_mont(a);
  fp_to_be48(out_sg48, fp_inv(m));
  fp_to_be48(out_fermat48, fp_inv_fermat(m));
}

// [k]P two ways: psi-decomposed Straus (g2_mul_u256_psi) and 255-bit double-and-add; 1 if they agree
extern "C" int hc_g2_mul_psi_check(const uint8_t* sig96, const uint32_t* k8) {
  G2A a;
  if (!g2_decompress(a, sig96, true)) return -1;
  G2J u = g2_mul_u256_psi(a, k8);
  G2J v = jac_mul_u256(jac_from_aff(a), k8);
  return jac_eq(u, v) ? 1 : 0;
}

// word-wise expand_message_xmd (32 B messages, host-built DST tail) against the byte-wise RFC 9380 path:
// 1 if the four hash_to_field elements agree
extern "C" int hc_h2f_xmd32_check(const uint8_t* msg32, const uint8_t* dst, uint32_t dl) {
  static XmdTail T;
  xmd_tail_build(T, dst, dl);
  Fp2 a[2], b[2];
  hash_to_field_xmd32(a, msg32, &T);
  hash_to_field_fp2x2(b, msg32, 32, dst, dl);
  return fp2_eq(a[0], b[0]) && fp2_eq(a[1], b[1]) ? 1 : 0;
}

// the phase pipeline of phases.h (k_h2c_p1 .. p4 with fp_pow_pm3d4_sos between) against the fused
// hash_to_g2_uncleared: 1 if the normalised points agree
extern "C" int hc_h2c_phases_check(const uint8_t* msg, uint32_t len, const uint8_t* dst, uint32_t dl) {
  static XmdTail T;
  xmd_tail_build(T, dst, dl);
  Fp2 u[2];
  if (len == 32)
    hash_to_field_xmd32(u, msg, &T);
  else
    hash_to_field_fp2x2(u, msg, len, dst, dl);
  H2cMap st[2];
  Fp e[2];
  h2c_p1(u, st, e);
  G2J q[2];
  for (int h = 0; h < 2; ++h) {
    Fp c;
    h2c_p2(st[h], e[h], fp_pow_pm3d4_sos(e[h]), c);
    q[h] = h2c_p3(st[h], c, fp_pow_pm3d4_sos(c));
  }
  G2A a = g2_to_aff(jac_add(q[0], q[1]));
  G2A b = g2_to_aff(hash_to_g2_uncleared(msg, len, dst, dl));
  return a.inf == b.inf && fp2_eq(a.x, b.x) && fp2_eq(a.y, b.y) ? 1 : 0;
}
// the decompression phases (k_dec_p1 .. p3) against g2_decompress: 1 if status and point agree
extern "C" int hc_dec_phases_check(const uint8_t* in96, int subgroup) {
  DecState ds;
  Fp e, c = fp_zero();
  G2A a{fp2_zero(), fp2_zero(), true};
  bool ok = dec_p1(in96, ds, e) == 0;
  if (ok && (ds.flags & DEC_PENDING)) {
    ok = dec_p2(ds, e, fp_pow_pm3d4_sos(e), c);
    if (ok) ok = dec_p3(ds, c, fp_pow_pm3d4_sos(c), subgroup != 0, a);
  }
  G2A b;
  bool okb = g2_decompress(b, in96, subgroup != 0);
  if (ok != okb) return 0;
  if (!ok) return 1;
  return a.inf == b.inf && (a.inf || (fp2_eq(a.x, b.x) && fp2_eq(a.y, b.y))) ? 1 : 0;
}

// the same product by the sign-aligned column form (GLV-SAC): 1 if it agrees with the branching psi-Straus
extern "C" int hc_g2_mul_sac_check(const uint8_t* sig96, const uint32_t* k8) {
  G2A a;
  if (!g2_decompress(a, sig96, true)) return -1;
  return jac_eq(g2_mul_u256_psi_sac(a, k8), g2_mul_u256_psi(a, k8)) ? 1 : 0;
}

// sum_i [d_i] P_i by the four-point sign-aligned column form (curve.h jac_msm4_sac), in G2 on four signatures
// and in G1 on four keys, against double-and-add per point; bit i of inf_mask replaces point i by the
// identity.  1 if both agree.
extern "C" int hc_msm4_check(const uint8_t* sigs384, const uint8_t* keys192, const uint64_t* d, uint32_t inf_mask) {
  G2J s[4], s_ref = jac_infinity<Fp2>();
  G1J x[4], x_ref = jac_infinity<Fp>();
  for (int i = 0; i < 4; ++i) {
    G2A a;
    G1A b;
    if (!g2_decompress(a, sigs384 + 96 * i, true) || !g1_decompress(b, keys192 + 48 * i, true)) return -1;
    s[i] = (inf_mask >> i) & 1 ? jac_infinity<Fp2>() : jac_from_aff(a);
    x[i] = (inf_mask >> i) & 1 ? jac_infinity<Fp>() : jac_from_aff(b);
    s_ref = jac_add(s_ref, jac_mul_u64(s[i], d[i]));
    x_ref = jac_add(x_ref, jac_mul_u64(x[i], d[i]));
  }
  return jac_eq(jac_msm4_sac(s, d), s_ref) && jac_eq(jac_msm4_sac(x, d), x_ref) ? 1 : 0;
}

// One affine pair addition of the MSM's affine levels (curve.h g2_aff_kind / g2_aff_den / g2_aff_sum, the inverse
// supplied as the batch inversion would) against the Jacobian addition.  mode 0: P + Q, 1: P + P, 2: P + (-P),
// 3: O + Q, 4: P + O, 5: O + O.  1 if both agree, -1 if a signature does not decode.
extern "C" int hc_aff_add_check(const uint8_t* sig_a, const uint8_t* sig_b, int mode) {
  G2A a, b;
  if (!g2_decompress(a, sig_a, false) || !g2_decompress(b, sig_b, false)) return -1;
  const G2A O{fp2_zero(), fp2_zero(), true};
  G2A p = a, q = b;
  if (mode == 1) q = a;
  if (mode == 2) q = G2A{a.x, fp2_neg(a.y), false};
  if (mode == 3 || mode == 5) p = O;
  if (mode == 4 || mode == 5) q = O;
  const uint32_t kind = g2_aff_kind(p, q);
  const Fp den = g2_aff_den(p, q, kind);
  const G2A r = g2_aff_sum(p, q, kind, fp_inv(den));
  const G2J want = jac_add(jac_from_aff(p), jac_from_aff(q));
  if (r.inf != jac_is_inf(want)) return 0;
  return jac_eq(jac_from_aff(r), want) ? 1 : 0;
}

// The LDS-form additions' exceptional cases (curve.h g2_madd_lds / g2_add_lds: a = q takes the tangent, a = -q gives
// the identity, inline), with the accumulator a rescaled Jacobian copy of a (Z != 1), against jac_add; mode 0 chord
// (a + b), 1 a + a, 2 a + (-a); `full` uses g2_add_lds with a Jacobian q.  1 if equal.
extern "C" int hc_lds_add_check(const uint8_t* sig_a, const uint8_t* sig_b, int mode, int full) {
  G2A a, b;
  if (!g2_decompress(a, sig_a, false) || !g2_decompress(b, sig_b, false)) return -1;
  G2A q = b;
  if (mode == 1) q = a;
  if (mode == 2) q = G2A{a.x, fp2_neg(a.y), false};
  const G2J aj = jac_dbl(jac_add(jac_from_aff(a), jac_from_aff(a)));  // 4a with Z != 1 ...
  G2J acc = jac_add(aj, jac_neg(jac_add(jac_from_aff(a), jac_dbl(jac_from_aff(a)))));  // ... minus 3a: a, Z != 1
  if (!jac_eq(acc, jac_from_aff(a)) || fp2_eq(acc.z, fp2_one())) return -2;
  const G2J want = jac_add(acc, jac_from_aff(q));
  if (full) {
    const G2J qj = jac_add(jac_dbl(jac_from_aff(q)), jac_neg(jac_from_aff(q)));  // q with Z != 1
    g2_add_lds(acc, qj);
  } else {
    g2_madd_lds(acc, q.x, q.y);
  }
  if (jac_is_inf(acc) != jac_is_inf(want)) return 0;
  return jac_eq(acc, want) ? 1 : 0;
}

// checks.h ck_in_subgroup (k_ck_sub: the LDS-accumulator form) against curve.h g2_in_subgroup_aff for the point
// decoded from in96 without a subgroup check (any point of E'(Fp2)); -1 if in96 is not on the curve, else the
// verdict (1 in G2, 0 not) when both agree, 2 when they differ
extern "C" int hc_ck_subgroup_check(const uint8_t* in96) {
  G2A a;
  if (!g2_decompress(a, in96, false) || a.inf) return -1;
  G2J slot;
  const bool x = ck_in_subgroup(a.x, a.y, slot), y = g2_in_subgroup_aff(a.x, a.y);
  return x != y ? 2 : (x ? 1 : 0);
}

// checks.h's split G2 sum of a group check (k_ck_tab_den / k_ck_tab_add levels with exact inverses, k_ck_sac's column
// loop, k_ck_bfin's affine form) against group_combine's g2_to_aff(jac_msm4_sac(...)).  sigs: 4 compressed G2 points
// (any may repeat, cancel or be the identity), rho: 4 coefficients, nl live members (rho and points past nl unused).
// 1 if equal.
extern "C" int hc_ck_g2_split_check(const uint8_t* sigs384, const uint64_t* rho_in, uint32_t nl) {
  G2AStore S[4];
  CkState c{};
  c.nl = nl;
  G2J sp[4];
  uint64_t rho[4];
  for (uint32_t m = 0; m < 4; ++m) {
    G2A a;
    if (!g2_decompress(a, sigs384 + 96 * m, false)) return -1;
    store_g2a(S[m], a);
    c.live[m] = m;
    sp[m] = m < nl ? jac_from_aff(a) : jac_infinity<Fp2>();
    rho[m] = m < nl ? rho_in[m] : 0;
  }
  G2A T[8];
  for (auto& t : T) t = G2A{fp2_zero(), fp2_zero(), true};
  auto getT = [&](uint32_t u) { return T[u]; };
  for (uint32_t l = 0; l < 3; ++l) {
    G2A out[3];
    uint32_t dsts[3];
    bool on[3] = {false, false, false};
    for (uint32_t e = 0; e < 3; ++e) {
      G2A A, B;
      if (!ck_tab_operands(l, e, c, S, getT, A, B, dsts[e])) continue;
      if (l == 0 && e == 0) T[0] = ck_member(c, S, 0);
      const uint32_t kind = g2_aff_kind(A, B);
      out[e] = g2_aff_sum(A, B, kind, fp_inv(g2_aff_den(A, B, kind)));
      on[e] = true;
    }
    for (uint32_t e = 0; e < 3; ++e)
      if (on[e]) T[dsts[e]] = out[e];
  }
  G2J acc;
  ck_sac_g2(rs_recode(rho), getT, acc);
  const G2A b = ck_g2_affine(acc, fp2_is_zero(acc.z) ? fp_zero() : fp_inv(fp2_norm(acc.z)));
  const G2A want = g2_to_aff(jac_msm4_sac(sp, rho));
  if (b.inf != want.inf) return 0;
  return b.inf || (fp2_eq(b.x, want.x) && fp2_eq(b.y, want.y)) ? 1 : 0;
}

// field.h fp2_mul_dig / fp2_sqr_dig (digit form, DG_FP2_DIG) against fp2_mul / fp2_sqr on n pseudo-random Fp2 pairs
// below p and the edge values 0, 1, p - 1; 1 if every product is equal
extern "C" int hc_fp2_mul_dig_check(uint64_t seed, uint32_t n) {
  uint64_t s = seed | 1;
  auto rnd = [&]() {
    Fp a;
    for (int i = 0; i < 12; ++i) {
      s ^= s << 13;
      s ^= s >> 7;
      s ^= s << 17;
      a.l[i] = (uint32_t)s;
    }
    a.l[11] &= 0x0fffffffu;  // below 2^380 < p
    return a;
  };
  Fp pm1 = fp_const(P_LIMBS);
  pm1.l[0] -= 1;
  const Fp edges[3] = {fp_zero(), fp_one(), pm1};
  for (uint32_t k = 0; k < n + 9; ++k) {
    Fp2 a, b;
    if (k < 9) {
      a = Fp2{edges[k % 3], edges[(k / 3) % 3]};
      b = Fp2{edges[(k + 1) % 3], pm1};
    } else {
      a = Fp2{rnd(), rnd()};
      b = Fp2{rnd(), rnd()};
    }
    const Fp2 x = fp2_mul_dig(a, b), y = fp2_mul(a, b);
    if (!fp2_eq(x, y)) return 0;
    if (!fp2_eq(fp2_mul_dig2(a, b), y) || !fp2_eq(fp2_mul_dig2(b, a), y)) return 0;
    if (!fp2_eq(fp2_sqr_dig(a), fp2_sqr(a)) || !fp2_eq(fp2_sqr_dig(b), fp2_sqr(b))) return 0;
    if (!fp2_eq(fp2_mul_dig<false>(a, b), y) || !fp2_eq(fp2_sqr_dig<false>(a), fp2_sqr(a))) return 0;
  }
  return 1;
}

// [k]P with the accumulator as a memory slot (curve.h g2_mul_u256_psi_lds, LDS on the device) against the
// register form; 1 if equal
extern "C" int hc_g2_mul_lds_check(const uint8_t* sig96, const uint32_t* k8) {
  G2A a;
  if (!g2_decompress(a, sig96, true)) return -1;
  G2J acc;
  g2_mul_u256_psi_lds(a, k8, acc);
  return jac_eq(acc, g2_mul_u256_psi(a, k8)) ? 1 : 0;
}

// fr.h lagrange_at_zero (64-bit plain chunks of the factors, quarter products) against rc_lambdas (one full
// Montgomery product per factor, one inversion for all t) for t distinct indices < 2^32 - 1.  1 if all equal.
extern "C" int hc_lagrange_check(const uint32_t* idx, uint32_t t) {
  std::vector<Fr> lam(t), pre(t);
  rc_lambdas(idx, t, lam.data(), pre.data());
  for (uint32_t j = 0; j < t; ++j) {
    const Fr l = lagrange_at_zero(idx, t, j);
    for (int w = 0; w < 8; ++w)
      if (l.l[w] != lam[j].l[w]) return 0;
  }
  return 1;
}

// Recover's per-round MSM (recover.h) on the host: lambdas with one Fr inversion (rc_lambdas) against
// lagrange_at_zero, the odd-multiple tables by the device's affine formulas (g2_aff_den / g2_aff_sum with exact
// inverses), the four wNAF schedules and the psi combination, against sum_j g2_mul_u256_psi(S_j, lambda_j).
// sigs: t compressed G2 points (any may be the identity), idx: t distinct share indices.  1 if equal.
extern "C" int hc_recover_msm_check(const uint8_t* sigs96, const uint32_t* idx, uint32_t t) {
  std::vector<Fr> lam(t), pre(t);
  rc_lambdas(idx, t, lam.data(), pre.data());
  std::vector<G2A> P(t);
  G2J want = jac_infinity<Fp2>();
  for (uint32_t j = 0; j < t; ++j) {
    if (!g2_decompress(P[j], sigs96 + 96 * j, false)) return -1;
    const Fr l = lagrange_at_zero(idx, t, j);
    for (int w = 0; w < 8; ++w)
      if (l.l[w] != lam[j].l[w]) return 0;
    want = jac_add(want, g2_mul_u256_psi(P[j], lam[j].l));
  }
  // tables: T[j][0] = P, D = 2P (tangent), T[j][e] = T[j][e-1] + D (chord)
  std::vector<G2A> T((size_t)t * RC_TAB);
  for (uint32_t j = 0; j < t; ++j) {
    if (P[j].inf) continue;
    const G2A d = g2_aff_sum(P[j], P[j], 2, fp_inv(g2_aff_den(P[j], P[j], 2)));
    T[(size_t)j * RC_TAB] = P[j];
    for (uint32_t e = 1; e < RC_TAB; ++e) {
      const G2A& a = T[(size_t)j * RC_TAB + e - 1];
      T[(size_t)j * RC_TAB + e] = g2_aff_sum(a, d, 1, fp_inv(g2_aff_den(a, d, 1)));
    }
  }
  // signed scalars (rc_signed), their digits, and the per-component signed digits (negated for a negated share)
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
  for (int i = 0; i < 4; ++i) {
    uint32_t tail;
    const uint32_t n = rc_schedule_naf(naf.data() + (size_t)i * t * RC_NAF, t, ev.data(), tail);
    if (n > t * RC_EV_PER_SHARE) return 0;
    G2JStore acc{fp2_zero(), fp2_zero(), fp2_zero()};
    for (uint32_t q = 0; q < n; ++q) {
      const uint32_t v = ev[q];
      for (uint32_t d = rc_ev_dbl(v); d > 0; --d) g2_dbl_lds(acc);
      const uint32_t j = rc_ev_j(v);
      if (P[j].inf) continue;
      const G2A& e = T[(size_t)j * RC_TAB + rc_ev_e(v)];
      g2_madd_lds(acc, e.x, rc_ev_neg(v) ? fp2_neg(e.y) : e.y);
    }
    for (uint32_t d = tail; d > 0; --d) g2_dbl_lds(acc);
    A[i] = G2J{acc.x, acc.y, acc.z};
  }
  return jac_eq(rc_combine(A[0], A[1], A[2], A[3]), want) ? 1 : 0;
}

// the width-5 signed digits of a 64-bit scalar evaluate back to it and keep their spacing; 1 if so
extern "C" int hc_wnaf_check(uint64_t d) {
  int8_t naf[RC_NAF];
  rc_wnaf(d, naf);
  unsigned __int128 v = 0;
  int last = -100;
  for (int b = (int)RC_NAF - 1; b >= 0; --b) {
    v = v * 2 + (__int128)naf[b];
    if (naf[b]) {
      if ((naf[b] & 1) == 0 || naf[b] > 15 || naf[b] < -15) return 0;
      if (last - b < (int)RC_W && last >= 0) return 0;
      last = b;
    }
  }
  return v == (unsigned __int128)d ? 1 : 0;
}

// Recover's divergent-round form (recover.h, k_rs_*) on the host: the sign-aligned tables by the device's three
// affine levels (exact inverses), the shared column loop over groups of RS_G shares, the even-d0 corrections and
// the sum of the group partial sums, against sum_j g2_mul_u256_psi(S_j, lambda_j).  1 if equal.
extern "C" int hc_recover_sac_check(const uint8_t* sigs96, const uint32_t* idx, uint32_t t) {
  std::vector<G2A> P(t);
  std::vector<RsDigits> dig(t);
  std::vector<G2A> T((size_t)t * 8);
  G2J want = jac_infinity<Fp2>();
  for (uint32_t j = 0; j < t; ++j) {
    if (!g2_decompress(P[j], sigs96 + 96 * j, false)) return -1;
    const Fr lam = lagrange_at_zero(idx, t, j);
    want = jac_add(want, g2_mul_u256_psi(P[j], lam.l));
    uint64_t d[4];
    rc_psi_digits(lam, d);
    dig[j] = rs_recode(d);
    if (P[j].inf) continue;
    Fp2 px[4], py[4];
    rs_points(P[j], px, py);
    T[(size_t)j * 8] = G2A{px[0], py[0], false};
    for (uint32_t l = 0; l < 3; ++l)
      for (uint32_t e = 0; e < 3; ++e) {
        uint32_t src, pb, dst;
        if (!rs_level(l, e, src, pb, dst)) continue;
        const G2A a = T[(size_t)j * 8 + src], b{px[pb], py[pb], false};
        if (fp2_eq(a.x, b.x)) return 0;  // no exceptional pair for P != O
        T[(size_t)j * 8 + dst] = g2_aff_sum(a, b, 1, fp_inv(g2_aff_den(a, b, 1)));
      }
  }
  G2J sum = jac_infinity<Fp2>();
  for (uint32_t j0 = 0; j0 < t; j0 += RS_G) {
    const uint32_t j1 = j0 + RS_G < t ? j0 + RS_G : t;
    G2JStore acc{fp2_zero(), fp2_zero(), fp2_zero()};
    for (int c = 64; c >= 0; --c) {
      if (c < 64) g2_dbl_lds(acc);
      for (uint32_t j = j0; j < j1; ++j) {
        if (P[j].inf) continue;
        const RsDigits& d = dig[j];
        const uint32_t e = c == 64 ? d.top
                                   : (uint32_t)((d.um[0] >> c) & 1u) | (uint32_t)((d.um[1] >> c) & 1u) << 1 |
                                         (uint32_t)((d.um[2] >> c) & 1u) << 2;
        const bool pos = c == 64 || ((d.sgn >> c) & 1u);
        const G2A& x = T[(size_t)j * 8 + e];
        g2_madd_lds(acc, x.x, pos ? x.y : fp2_neg(x.y));
      }
    }
    for (uint32_t j = j0; j < j1; ++j)
      if (!P[j].inf && dig[j].even) g2_madd_lds(acc, T[(size_t)j * 8].x, fp2_neg(T[(size_t)j * 8].y));
    sum = jac_add(sum, G2J{acc.x, acc.y, acc.z});
  }
  return jac_eq(sum, want) ? 1 : 0;
}


// cyc_exp_z (Karabina compressed squarings, batched decompression) against the Granger-Scott square-and-multiply
// chain, on n cyclotomic elements f^((p^6 - 1)(p^2 + 1)) of pseudo-random f, plus the element 1 (every
// denominator zero: the uncompressed fallback).  Returns the number of mismatches.
extern "C" int hc_cyc_exp_check(uint64_t seed, uint32_t n) {
  uint64_t s = seed | 1;
  auto rnd_fp = [&s]() {
    Fp a;
    for (int i = 0; i < 12; i += 2) {
      s ^= s << 13;
      s ^= s >> 7;
      s ^= s << 17;
      a.l[i] = (uint32_t)s;
      a.l[i + 1] = (uint32_t)(s >> 32);
    }
    a.l[11] &= 0x1fffffffu;
    return fp_reduce_once(fp_reduce_once(fp_reduce_once(a)));
  };
  auto gs = [](const Fp12& a) {
    Fp12 acc = a;
    for (int b = 62; b >= 0; --b) {
      acc = fp12_cyc_sqr(acc);
      if ((Z_ABS >> b) & 1) acc = fp12_mul(acc, a);
    }
    return fp12_conj(acc);
  };
  int bad = 0;
  for (uint32_t it = 0; it <= n; ++it) {
    Fp12 f2 = fp12_one();
    if (it < n) {
      Fp12 f;
      Fp* c[12] = {&f.c0.c0.c0, &f.c0.c0.c1, &f.c0.c1.c0, &f.c0.c1.c1, &f.c0.c2.c0, &f.c0.c2.c1,
                   &f.c1.c0.c0, &f.c1.c0.c1, &f.c1.c1.c0, &f.c1.c1.c1, &f.c1.c2.c0, &f.c1.c2.c1};
      for (int i = 0; i < 12; ++i) *c[i] = rnd_fp();
      const Fp12 f1 = fp12_mul(fp12_conj(f), fp12_inv(f));
      f2 = fp12_mul(fp12_frob(fp12_frob(f1)), f1);
    }
    const Fp12 x = cyc_exp_z(f2), y = gs(f2);
    const Fp6* u[2] = {&x.c0, &x.c1};
    const Fp6* v[2] = {&y.c0, &y.c1};
    bool eq = true;
    for (int h = 0; h < 2; ++h)
      eq = eq && fp2_eq(u[h]->c0, v[h]->c0) && fp2_eq(u[h]->c1, v[h]->c1) && fp2_eq(u[h]->c2, v[h]->c2);
    bad += !eq;
  }
  return bad;
}

// Recover's pairing-check pipeline (checks.h) step for step on the host against pair_check's formula
// (final_exp_cubed(miller_loop<2>)): the per-round lines of Q1 (unevaluated, ck_lines) evaluated at P1, the lines of
// Q2 at -g1, the easy part through ck_fe1 / ck_inv with the Fp inversion of the batch, the hard part through the
// compressed chains (ck_expsq / ck_expdec, or ck_exp_plain where a denominator is zero) and ck_mul_op.  `np` drops
// pairs as pair_check does (bit 0: (P1, Q1), bit 1: (-g1, Q2)).  Returns 1 when both Fp12 values are equal.
static bool g_split_bad = false;  // ck_cyc_half disagreed with cyc_sqr_c (hc_ck_pipeline_check returns 4)
static Fp12 hc_ck_expz(const Fp12& x, const Fp12* y, uint32_t nfrob, uint32_t conj) {
  // k_ck_expsq, k_ck_expdec (norms inverted in the lane by ck_inv6), k_ck_explain; times op(y) when given
  CycC sn[CK_NPOW];
  Fp nv[CK_NPOW];
  Fp12 xz;
  if (fp12_is_one(x)) {
    xz = fp12_one();
  } else if (ck_expsq(x, [&](int i, const CycC& c, const Fp& n) { sn[i] = c; nv[i] = n; })) {
    xz = ck_exp_plain(x);
  } else {
    // k_ck_expsq2: the two halves of the split squaring (ck_cyc_half), outputs swapped after every step
    Fp2 u0 = x.c1.c0, v0 = x.c0.c2, u1 = x.c0.c1, v1 = x.c1.c2;
    int n = 0;
    for (int k = 1; k <= 63; ++k) {
      Fp2 a0, b0, a1, b1;
      ck_cyc_half(0, u0, v0, u1, v1, a0, b0);
      ck_cyc_half(1, u1, v1, u0, v0, a1, b1);
      u0 = a0, v0 = b0, u1 = a1, v1 = b1;
      if ((Z_ABS >> k) & 1) {
        if (!fp2_eq(u0, sn[n].g2) || !fp2_eq(v0, sn[n].g3) || !fp2_eq(u1, sn[n].g4) || !fp2_eq(v1, sn[n].g5))
          g_split_bad = true;
        ++n;
      }
    }
    ck_inv6([&](int i) { return nv[i]; }, [&](int i, const Fp& v) { nv[i] = v; });
    xz = ck_expdec([&](int i, CycC& c, Fp& n) { c = sn[i]; n = nv[i]; });
  }
  return y ? ck_mul_op(xz, *y, nfrob, conj) : xz;
}
extern "C" int hc_ck_pipeline_check(const uint8_t* pk48, const uint8_t* q1_96, const uint8_t* q2_96, int np) {
  G1A p1;
  G2A q1, q2;
  if (!g1_decompress(p1, pk48, true) || !g2_decompress(q1, q1_96, false) || !g2_decompress(q2, q2_96, false)) return -1;
  G1A P[2];
  G2A Q[2];
  int n = 0;
  if (np & 1) { P[n] = p1; Q[n] = q1; ++n; }
  if (np & 2) { P[n] = G1A{fp_const(G1_GEN_X), fp_const(G1_GEN_NEG_Y), false}; Q[n] = q2; ++n; }
  const Fp12 ref = n ? final_exp_cubed(miller_loop<2>(P, Q, n)) : fp12_one();
  std::vector<CkLine> l1(CK_STEPS), l2(CK_STEPS);
  ck_lines(q1.x, q1.y, [&](uint32_t s, const CkLine& l) { l1[s] = l; });
  ck_lines(q2.x, q2.y, [&](uint32_t s, const CkLine& l) { l2[s] = l; });
  const Fp12 f = ck_miller((uint32_t)np, p1.x, p1.y, [&](uint32_t s, uint32_t pair) { return pair ? l2[s] : l1[s]; });
  {
    const Fp2* u[6] = {&f.c0.c0, &f.c0.c1, &f.c0.c2, &f.c1.c0, &f.c1.c1, &f.c1.c2};
    // k_ck_miller's digit-form loop with the accumulator in a column (fpd.h; bounds asserted: DG_FD_CHECK)
    uint32_t col[144];
    Fd12Col<1> fc{col};
    const Fp12 fl =
        ck_miller_col((uint32_t)np, p1.x, p1.y, [&](uint32_t s, uint32_t pair) { return pair ? l2[s] : l1[s]; }, fc);
    const Fp2* w[6] = {&fl.c0.c0, &fl.c0.c1, &fl.c0.c2, &fl.c1.c0, &fl.c1.c1, &fl.c1.c2};
    for (int i = 0; i < 6; ++i)
      if (!fp2_eq(*u[i], *w[i])) return 9;
    if (g_fd_bad) return 7;
  }
  // each pair in a lane of its own (its own squarings; xr.h k_xg_miller), the two values multiplied by k_ck_easy
  const Fp12 m0 = (np & 1) ? ck_miller1(p1.x, p1.y, [&](uint32_t s) { return l1[s]; }) : fp12_one();
  const Fp12 m1 = (np & 2) ? ck_miller1(fp_const(G1_GEN_X), fp_const(G1_GEN_NEG_Y), [&](uint32_t s) { return l2[s]; })
                           : fp12_one();
  const Fp12 f01 = fp12_mul(m0, m1);
  {
    // xr.h k_xg_miller: each pair's lines computed in the lane (ck_miller1_fly), the same values as from the tables
    G2Proj T;
    const Fp12 w0 = (np & 1) ? ck_miller1_fly([&]() { return q1; }, p1.x, p1.y, T) : fp12_one();
    const Fp12 w1 =
        (np & 2) ? ck_miller1_fly([&]() { return q2; }, fp_const(G1_GEN_X), fp_const(G1_GEN_NEG_Y), T) : fp12_one();
    const Fp2* u[12] = {&m0.c0.c0, &m0.c0.c1, &m0.c0.c2, &m0.c1.c0, &m0.c1.c1, &m0.c1.c2,
                        &m1.c0.c0, &m1.c0.c1, &m1.c0.c2, &m1.c1.c0, &m1.c1.c1, &m1.c1.c2};
    const Fp2* v[12] = {&w0.c0.c0, &w0.c0.c1, &w0.c0.c2, &w0.c1.c0, &w0.c1.c1, &w0.c1.c2,
                        &w1.c0.c0, &w1.c0.c1, &w1.c0.c2, &w1.c1.c0, &w1.c1.c1, &w1.c1.c2};
    for (int i = 0; i < 12; ++i)
      if (!fp2_eq(*u[i], *v[i])) return 8;
  }
  {
    const Fp2* u[6] = {&f.c0.c0, &f.c0.c1, &f.c0.c2, &f.c1.c0, &f.c1.c1, &f.c1.c2};
    const Fp2* v[6] = {&f01.c0.c0, &f01.c0.c1, &f01.c0.c2, &f01.c1.c0, &f01.c1.c1, &f01.c1.c2};
    for (int i = 0; i < 6; ++i)
      if (!fp2_eq(*u[i], *v[i])) return 3;
  }
  // k_ck_easy
  CkInv inv;
  const Fp nt = ck_fe1(f, inv);
  const Fp12 f1 = ck_mul_op(ck_inv(f, inv, fp_inv(nt)), f, 0, 1);
  const Fp12 f2 = ck_mul_op(f1, f1, 2, 0);
  // the five x^z with their next factors (drand_gpu.hip run_checks), k_ck_final
  const Fp12 t0 = hc_ck_expz(f2, &f2, 0, 1);
  const Fp12 t1 = hc_ck_expz(t0, &t0, 0, 1);
  const Fp12 a = hc_ck_expz(t1, &t1, 1, 0);
  const Fp12 t = hc_ck_expz(hc_ck_expz(a, nullptr, 0, 0), &a, 2, 0);
  const Fp12 c = ck_mul_op(ck_mul_op(f2, f2, 0, 0), f2, 0, 0);
  const Fp12 res = n ? ck_mul_op(ck_mul_op(t, a, 0, 1), c, 0, 0) : fp12_one();
  if (g_split_bad) return 4;
  const Fp2* u[6] = {&res.c0.c0, &res.c0.c1, &res.c0.c2, &res.c1.c0, &res.c1.c1, &res.c1.c2};
  const Fp2* v[6] = {&ref.c0.c0, &ref.c0.c1, &ref.c0.c2, &ref.c1.c0, &ref.c1.c1, &ref.c1.c2};
  for (int i = 0; i < 6; ++i)
    if (!fp2_eq(*u[i], *v[i])) return 0;
  return 1;
}

// xr.h xq_sum4 (the cross-round quad sums of k_xq_sum: an affine 8-entry table built in three levels with one Fp
// inversion per level, the column loop) against sum_i [rho_i] P_i by double-and-add.  sigs: 4 compressed G2 points
// (repeats, negations and the identity allowed), rho: 4 coefficients, members past nl are the identity (rho 0).
extern "C" int hc_xq_sum_check(const uint8_t* sigs384, const uint64_t* rho_in, uint32_t nl) {
  G2A P[4];
  uint64_t rho[4];
  G2J ref = jac_infinity<Fp2>();
  for (uint32_t m = 0; m < 4; ++m) {
    if (!g2_decompress(P[m], sigs384 + 96 * m, false)) return -1;
    if (m >= nl) P[m] = G2A{fp2_zero(), fp2_zero(), true};
    rho[m] = m < nl ? rho_in[m] : 0;
    ref = jac_add(ref, jac_mul_u64(jac_from_aff(P[m]), rho[m]));
  }
  G2A T[8];
  for (auto& t : T) t = G2A{fp2_zero(), fp2_zero(), true};
  G2J acc;
  xq_sum4([&](uint32_t m) { return P[m]; }, rho, [&](uint32_t u) { return T[u]; },
          [&](uint32_t u, const G2A& t) { T[u] = t; }, acc);
  return jac_eq(acc, ref) ? 1 : 0;
}

// fpd.h against field.h: the digit-form Fp12 squaring and sparse line product on random elements and on the extreme one
// (every component p - 1), bounds asserted.  Returns the number of mismatches (+1000 on a bound violation).
extern "C" int hc_fd_check(uint64_t seed, int n) {
  uint64_t st = seed * 0x9e3779b97f4a7c15ull + 1;
  auto rnd = [&]() {
    st ^= st << 13;
    st ^= st >> 7;
    st ^= st << 17;
    return st;
  };
  auto rfp = [&](bool top) {
    Fp a;
    if (top) {
      a = fp_const(FP_ONE);
      a = fp_sub(fp_zero(), a);  // p - R mod p: a large value
      for (int i = 0; i < 12; ++i) a.l[i] = i < 11 ? 0xffffffffu : a.l[i];
      return fp_reduce_once(fp_reduce_once(a));
    }
    for (int i = 0; i < 12; ++i) a.l[i] = (uint32_t)rnd();
    a.l[11] &= 0x0fffffffu;
    return fp_reduce_once(fp_reduce_once(fp_reduce_once(a)));
  };
  int bad = 0;
  g_fd_bad = false;
  for (int t = 0; t < n; ++t) {
    const bool top = t == 0;
    Fp12 a;
    Fp* c[12] = {&a.c0.c0.c0, &a.c0.c0.c1, &a.c0.c1.c0, &a.c0.c1.c1, &a.c0.c2.c0, &a.c0.c2.c1,
                 &a.c1.c0.c0, &a.c1.c0.c1, &a.c1.c1.c0, &a.c1.c1.c1, &a.c1.c2.c0, &a.c1.c2.c1};
    for (int i = 0; i < 12; ++i) *c[i] = rfp(top);
    const Fp2 l0{rfp(top), rfp(top)}, l1{rfp(top), rfp(top)}, l4{rfp(top), rfp(top)};
    const Fp12 s1 = fp12_sqr(a), s2 = fd12_to(fd12_sqr(fd12_from(a)));
    const Fp12 m1 = fp12_mul_014(a, l0, l1, l4);
    const Fp12 m2 = fd12_to(fd12_mul_014(fd12_from(a), fd2_from(l0), fd2_from(l1), fd2_from(l4)));
    // chained: the reduced outputs of one operation as the next one's inputs
    const Fp12 q1 = fp12_mul_014(fp12_sqr(s1), l0, l1, l4);
    const Fp12 q2 = fd12_to(fd12_mul_014(fd12_sqr(fd12_sqr(fd12_from(a))), fd2_from(l0), fd2_from(l1), fd2_from(l4)));
    // fd2_mul (two reductions, signed c0 columns) against fd2_mul3 (three), operands up to 40 p
    for (int sc : {1, 7, 40}) {
      auto big = [&](const Fp& v) {
        const Fd r = fd_from(v);
        Fd acc = r;
        for (int i = 1; i < sc; ++i) acc = fd_add(acc, r);
        return acc;
      };
      const Fd2 a2{big(rfp(top)), big(rfp(false))}, b2{big(rfp(false)), big(rfp(top))};
      bad += !fp2_eq(fd2_to(fd2_mul(a2, b2)), fd2_to(fd2_mul3(a2, b2)));
      bad += !fp2_eq(fd2_to(fd2_mul(b2, a2)), fd2_to(fd2_mul3(a2, b2)));
    }
    const Fp12* x[3] = {&s1, &m1, &q1};
    const Fp12* y[3] = {&s2, &m2, &q2};
    for (int k = 0; k < 3; ++k) {
      const Fp2* u[6] = {&x[k]->c0.c0, &x[k]->c0.c1, &x[k]->c0.c2, &x[k]->c1.c0, &x[k]->c1.c1, &x[k]->c1.c2};
      const Fp2* v[6] = {&y[k]->c0.c0, &y[k]->c0.c1, &y[k]->c0.c2, &y[k]->c1.c0, &y[k]->c1.c1, &y[k]->c1.c2};
      bool eq = true;
      for (int i = 0; i < 6; ++i) eq = eq && fp2_eq(*u[i], *v[i]);
      bad += !eq;
    }
  }
  return bad + (g_fd_bad ? 1000 : 0);
}
