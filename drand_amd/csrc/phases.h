// Phase kernels of hash-to-G2 (A9) and sigma decompression (A10).
//
// Both are dominated by Fp exponentiations x^((p-3)/4): four per round in hash-to-G2 (two per simplified
// SWU map: the norm root and the root of (g0 + s)/2), two per item in the decompression.  Fused into one
// lane-per-item kernel, the exponentiation chain shares the register file with everything else the item
// keeps live (the SWU / isogeny state, the SHA-256 expansion, the Fp2 tower temporaries), the kernel sits
// at 256 VGPRs with ~2 KB of scratch per lane, and at 100k rounds 1563 waves leave half the SIMDs with one
// wave.  Here each item runs as a pipeline of short kernels whose state lives in HBM between them (a few
// hundred bytes per item, microseconds of traffic against milliseconds of arithmetic), and every
// exponentiation of the batch -- both maps of every round, both roots of every signature -- goes through
// one register-lean kernel, k_exp_pm3d4 (SOS products in the radix-2^28 digit form, no calls, no scratch).
//
//   hash-to-G2 (per batch of R rounds, M = 2R map items):
//     k_h2c_p1a (R)  expand_message_xmd, both u_h, den_h, norm(den_0 den_1)
//     k_binv_*       1 / norm(den_0 den_1) for every round: Montgomery's trick across the batch
//     k_h2c_p1b (R)  x1 = -B/A (1 + 1/den) for both maps, gx1; exponent input norm(gx1)
//     k_exp     (M)  t = norm(gx1)^((p-3)/4)
//     k_h2c_p2  (M)  s1 = t n1, square test, x / g / s of the chosen branch; input c of the second root
//     k_exp     (M)  t2 = c^((p-3)/4)
//     k_h2c_p3  (M)  y = sqrt(g) from c, t2 (checked; the full root as a fallback), sgn0 fix, 3-isogeny
//     k_h2c_p4a (R)  q0 + q1 (Jacobian), norm(Z)
//     k_binv_*       1 / norm(Z) for every round
//     k_h2c_p4b (R)  normalised to Z = 1
//   sigma decompression (per batch of N items):
//     k_dec_p1  (N)  flags, canonical x, rhs = x^3 + 4(1+u); exponent input norm(rhs)
//     k_exp     (N)
//     k_dec_p2  (N)  norm root (not a square: not on the curve), input c of the second root
//     k_exp     (N)
//     k_dec_p3  (N)  y, sign flag, optional subgroup check, (round, key) cell claim
// Every value is the one the fused code (h2c.h sswu_g2 / iso_map_g2, curve.h g2_decompress) computes: the
// square roots are unique up to sign and the sign is fixed by sgn0 / the flag bit.
#pragma once

namespace dg {

struct H2cMap {
  Fp2 u, x, g;  // field element, x-coordinate and g(x) on E2' of one simplified-SWU map
};
struct DecState {
  Fp2 x, g;        // x and rhs = x^3 + b'
  uint32_t flags;  // DEC_* below
  uint32_t pad[3];
};
constexpr uint32_t DEC_PENDING = 1, DEC_SIGN = 2, DEC_INF = 4;
constexpr uint32_t BINV_C = 32;  // chunk of the batch inversion (k_binv_*)
#ifndef DG_BINV_K
#define DG_BINV_K 8  // 4: C3 816 / 814 k against 826 / 820 k at 8 (one root launch up to 4.2 M values), headline equal
#endif
constexpr uint32_t BINV_T = 256, BINV_K = DG_BINV_K;  // block-tree batch inversion (k_binv_blk_*): lanes x values per lane
constexpr uint32_t BINV_R = 8;                // values per lane of the single-workgroup root inversion

// ------------------------------------------------------------------------------ exponentiation
// x^((p-3)/4) by a width-4 sliding-window schedule (the 8 odd powers x, x^3, .., x^15; 376 squarings and 85
// multiplications instead of 378 and 108 at width 3; tools/microbench/expchain.hip: -7%), SOS products in the
// digit form.  The schedule is wave-uniform (scalar loads), the table entry is picked by a v_cndmask chain.
DGI Fp fp_pow_pm3d4_sos(const Fp& x) {
  // eight separately named entries, built and read with constant indices only: a table array whose build
  // loop the compiler leaves rolled is indexed at run time and lives in scratch (10x the kernel's traffic)
  uint32_t t0[14], t1[14], t2[14], t3[14], t4[14], t5[14], t6[14], t7[14], x2[14], acc[14], nxt[14], m[14];
  fp28_unpack(x.l, t0);
  DG_COUNT_SQR();
  fp28_sos_sqr_d(t0, x2);
  DG_COUNT_MUL();
  fp28_sos_mul_d(t0, x2, t1);
  DG_COUNT_MUL();
  fp28_sos_mul_d(t1, x2, t2);
  DG_COUNT_MUL();
  fp28_sos_mul_d(t2, x2, t3);
  DG_COUNT_MUL();
  fp28_sos_mul_d(t3, x2, t4);
  DG_COUNT_MUL();
  fp28_sos_mul_d(t4, x2, t5);
  DG_COUNT_MUL();
  fp28_sos_mul_d(t5, x2, t6);
  DG_COUNT_MUL();
  fp28_sos_mul_d(t6, x2, t7);
  // m = t[q] for a wave-uniform q (v_cndmask chain; the empty asm keeps the chain from being folded into
  // a load through a selected pointer)
  auto pick = [&](int q) {
#pragma unroll
    for (int d = 0; d < 14; ++d) {
      uint32_t e[8] = {t0[d], t1[d], t2[d], t3[d], t4[d], t5[d], t6[d], t7[d]};
#pragma unroll
      for (int j = 0; j < 8; ++j) DG_PIN(e[j]);
      uint32_t v = e[0];
#pragma unroll
      for (int j = 1; j < 8; ++j) v = q == j ? e[j] : v;
      m[d] = v;
    }
  };
  pick(EXP_PM3D4_W4_FIRST);
#pragma unroll
  for (int d = 0; d < 14; ++d) acc[d] = m[d];
  for (int s = 0; s < EXP_PM3D4_W4_NSTEPS; ++s) {
    const int k = EXP_PM3D4_W4_STEPS[s][0];
    const int idx = EXP_PM3D4_W4_STEPS[s][1];
    for (int j = 0; j < k; ++j) {
      DG_COUNT_SQR();
      fp28_sos_sqr_d(acc, nxt);
#pragma unroll
      for (int d = 0; d < 14; ++d) acc[d] = nxt[d];
    }
    if (idx >= 0) {
      pick(idx);
      DG_COUNT_MUL();
      fp28_sos_mul_d(acc, m, nxt);
#pragma unroll
      for (int d = 0; d < 14; ++d) acc[d] = nxt[d];
    }
  }
  Fp r;
  fp28_pack(acc, r.l);
  return fp_reduce_once(r);
}

// ------------------------------------------------------------------------------ shared square-root tail
// The second half of the Fp2 square root of fp2_sqrt_with_norm_root (field.h): c = (a0 + s)/2 (or a0 when
// a1 = 0, which makes the same formula return sqrt(a0) or sqrt(-a0) u), t = c^((p-3)/4).  Returns whether
// r^2 == a.
DGI Fp sqrt_c_input(const Fp2& a, const Fp& s) {
  return fp_is_zero(a.c1) ? a.c0 : fp_mul(fp_add(a.c0, s), fp_const(FP_TWO_INV));
}
DGI bool sqrt_finish(Fp2& r, const Fp2& a, const Fp& c, const Fp& t) {
  Fp ct = fp_mul(c, t);
  Fp at2 = fp_mul(fp_mul(a.c1, t), fp_const(FP_TWO_INV));
  bool c_square = fp_eq(fp_mul(ct, t), fp_one());
  r = Fp2{fp_sel(c_square, at2, ct), fp_sel(c_square, fp_neg(ct), at2)};
  return fp2_eq(fp2_sqr(r), a);
}

// rare paths kept out of line so their exponentiations do not inflate the phase kernels' registers
DGN bool fp2_sqrt_slow(Fp2& r, const Fp2& a) { return fp2_sqrt(r, a); }
DGN bool g2_in_subgroup_slow(const Fp2& x, const Fp2& y) { return g2_in_subgroup_aff(x, y); }

// ------------------------------------------------------------------------------ hash-to-G2 phases
// P1 of round r, split around a batch inversion (Montgomery's trick across the batch, k_binv_*: one
// safegcd per ~10^5 rounds instead of one per round).  p1a: den_h of both maps (kept in st[h].x) and the
// norm of D = d_0 d_1 (d_h = den_h, or 1 when den_h = 0), the value to invert.
DGI void h2c_p1a(const Fp2 (&u)[2], H2cMap (&st)[2], Fp& nD) {
  const Fp2 Z = fp2_const(SSWU_Z);
  Fp2 d[2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    Fp2 zu2 = fp2_mul(Z, fp2_sqr(u[h]));
    Fp2 den = fp2_add(fp2_sqr(zu2), zu2);
    st[h].u = u[h];
    st[h].x = den;
    d[h] = fp2_is_zero(den) ? fp2_one() : den;
  }
  nD = fp2_norm(fp2_mul(d[0], d[1]));
}
// p1b: with inv_nD = 1 / norm(D): 1/den_h, x1 = -B/A (1 + 1/den) (B/(ZA) when den = 0), gx1 and the first
// exponent inputs norm(gx1)
DGI void h2c_p1b(H2cMap (&st)[2], const Fp& inv_nD, Fp (&ein)[2]) {
  const Fp2 A = fp2_const(SSWU_A), B = fp2_const(SSWU_B);
  bool zero[2];
  Fp2 d[2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    zero[h] = fp2_is_zero(st[h].x);
    d[h] = zero[h] ? fp2_one() : st[h].x;
  }
  Fp2 D = fp2_mul(d[0], d[1]);
  Fp2 inv = Fp2{fp_mul(D.c0, inv_nD), fp_neg(fp_mul(D.c1, inv_nD))};  // fp2_inv(D)
  Fp2 inv_h[2] = {fp2_mul(inv, d[1]), fp2_mul(inv, d[0])};
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    Fp2 x1 = zero[h] ? fp2_const(SSWU_B_OVER_ZA) : fp2_mul(fp2_const(SSWU_MINUS_B_OVER_A), fp2_add(fp2_one(), inv_h[h]));
    Fp2 gx1 = fp2_add(fp2_mul(fp2_add(fp2_sqr(x1), A), x1), B);
    st[h].x = x1;
    st[h].g = gx1;
    ein[h] = fp2_norm(gx1);
  }
}
// the fused form (host checks, opcounts): both halves around one inversion
DGI void h2c_p1(const Fp2 (&u)[2], H2cMap (&st)[2], Fp (&ein)[2]) {
  Fp nD;
  h2c_p1a(u, st, nD);
  h2c_p1b(st, fp_inv(nD), ein);
}
// P2 of one map: t = n1^((p-3)/4); the branch of sswu_g2 (h2c.h) and the input c of the second root
DGI void h2c_p2(H2cMap& st, const Fp& n1, const Fp& t, Fp& c) {
  const Fp2 A = fp2_const(SSWU_A), B = fp2_const(SSWU_B), Z = fp2_const(SSWU_Z);
  Fp s1 = fp_mul(t, n1);  // n1^((p+1)/4)
  bool sq1 = fp_eq(fp_sqr(s1), n1);
  Fp s = s1;
  if (!sq1) {
    Fp2 zu2 = fp2_mul(Z, fp2_sqr(st.u));
    st.x = fp2_mul(zu2, st.x);
    st.g = fp2_add(fp2_mul(fp2_add(fp2_sqr(st.x), A), st.x), B);
    // s1^2 = -n1 ; norm(gx2) = 5^3 norm(u)^6 n1 ; sqrt = norm(u)^3 * 5 * sqrt(-5) * s1
    Fp nu = fp2_norm(st.u);
    Fp nu3 = fp_mul(fp_sqr(nu), nu);
    s = fp_mul(fp_mul(nu3, fp_small(5)), fp_mul(fp_const(FP_SQRT_MINUS5), s1));
  }
  c = sqrt_c_input(st.g, s);
}
// P3 of one map: y = sqrt(g), its sign by sgn0(u), then the 3-isogeny (Jacobian, no inversion)
DGI G2J h2c_p3(const H2cMap& st, const Fp& c, const Fp& t) {
  Fp2 y;
  if (!sqrt_finish(y, st.g, c, t)) fp2_sqrt_slow(y, st.g);  // never taken for a square g
  if (fp2_sgn0(st.u) != fp2_sgn0(y)) y = fp2_neg(y);
  return iso_map_g2(st.x, y);
}

// ------------------------------------------------------------------------------ decompression phases
// P1: flags and x of a 96 B encoding; returns the status; exponent input norm(x^3 + b')
DGI uint8_t dec_p1(const uint8_t* in, DecState& ds, Fp& ein) {
  ds.flags = 0;
  ein = fp_zero();
  const uint8_t f = in[0];
  if (!(f & 0x80)) return 2;
  if (f & 0x40) {
    if (f != 0xc0) return 2;
    uint32_t o = 0;
    for (int i = 1; i < 96; ++i) o |= in[i];
    if (o) return 2;
    ds.flags = DEC_INF;
    return 0;
  }
  uint8_t b[48];
  for (int i = 0; i < 48; ++i) b[i] = in[i];
  b[0] &= 0x1f;
  Fp x1, x0;
  if (!fp_from_be48_plain(x1, b)) return 2;
  if (!fp_from_be48_plain(x0, in + 48)) return 2;
  ds.x = Fp2{fp_to_mont(x0), fp_to_mont(x1)};
  ds.g = fp2_add(fp2_mul(fp2_sqr(ds.x), ds.x), fp2_const(FP2_B_G2));
  ds.flags = DEC_PENDING | ((f & 0x20) ? DEC_SIGN : 0u);
  ein = fp2_norm(ds.g);
  return 0;
}
// P2: the norm root; false when rhs is not a square (x is not on the curve); the second exponent input
DGI bool dec_p2(const DecState& ds, const Fp& n, const Fp& t, Fp& c) {
  Fp s = fp_mul(t, n);
  if (!fp_eq(fp_sqr(s), n)) return false;
  c = sqrt_c_input(ds.g, s);
  return true;
}
// P3: y and its sign; false if no root (never for a square rhs) or outside G2 when `subgroup`
DGI bool dec_p3(const DecState& ds, const Fp& c, const Fp& t, bool subgroup, G2A& out) {
  Fp2 y;
  if (!sqrt_finish(y, ds.g, c, t) && !fp2_sqrt_slow(y, ds.g)) return false;
  if (((ds.flags & DEC_SIGN) != 0) != fp2_lex_largest(y)) y = fp2_neg(y);
  out = G2A{ds.x, y, false};
  if (subgroup && !g2_in_subgroup_slow(ds.x, y)) return false;
  return true;
}

#if defined(__HIP__)
// x^((p-3)/4) with the width-3 table (x, x^3, x^5, x^7) in LDS (DG_EXP_LDS=1, an A/B of k_exp_pm3d4): without the
// table in registers the kernel fits 3 waves per SIMD (168 VGPRs) instead of 2, the four entries packed (12 limbs,
// 48 B) lane-major in LDS, 192 B per lane, 147 KB per CU at 3 waves per SIMD; 378 squarings and 108 products
// instead of 376 and 85
#ifndef DG_EXP_LDS
#define DG_EXP_LDS 0
#endif
// DG_EXP_LDS=2: the width-2 table (x, x^3; 96 B per lane) at 4 waves per SIMD, 378 squarings and 142 products
#if DG_EXP_LDS == 2
#define DG_EXP_NTAB 2
#define DG_EXP_SCHED(f) EXP_PM3D4_W2_##f
#else
#define DG_EXP_NTAB 4
#define DG_EXP_SCHED(f) EXP_PM3D4_##f
#endif
#if DG_EXP_LDS
DGI void fp_pow_pm3d4_lds(const Fp& x, Fp& out, uint32_t* tab, uint32_t stride) {
  // tab[(e * 12 + l) * stride]: limb l of entry e of this lane (stride = threads per block)
  uint32_t t[14], x2[14], acc[14], nxt[14], m[14];
  fp28_unpack(x.l, t);
  fp28_sos_sqr_d(t, x2);
  auto put = [&](int e, const uint32_t (&d)[14]) {
    uint32_t w[12];
    fp28_pack(d, w);
#pragma unroll
    for (int l = 0; l < 12; ++l) tab[(e * 12 + l) * stride] = w[l];
  };
  auto get = [&](int e, uint32_t (&d)[14]) {
    uint32_t w[12];
#pragma unroll
    for (int l = 0; l < 12; ++l) w[l] = tab[(e * 12 + l) * stride];
    fp28_unpack(w, d);
  };
  put(0, t);
#pragma unroll 1
  for (int e = 1; e < DG_EXP_NTAB; ++e) {
    fp28_sos_mul_d(t, x2, nxt);
#pragma unroll
    for (int d = 0; d < 14; ++d) t[d] = nxt[d];
    put(e, t);
  }
  get(DG_EXP_SCHED(FIRST), acc);
  for (int s = 0; s < DG_EXP_SCHED(NSTEPS); ++s) {
    const int k = DG_EXP_SCHED(STEPS)[s][0];
    const int idx = DG_EXP_SCHED(STEPS)[s][1];
    for (int j = 0; j < k; ++j) {
      fp28_sos_sqr_d(acc, nxt);
#pragma unroll
      for (int d = 0; d < 14; ++d) acc[d] = nxt[d];
    }
    if (idx >= 0) {
      get(idx, m);
      fp28_sos_mul_d(acc, m, nxt);
#pragma unroll
      for (int d = 0; d < 14; ++d) acc[d] = nxt[d];
    }
  }
  Fp r;
  fp28_pack(acc, r.l);
  out = fp_reduce_once(r);
}
#endif
#ifndef DG_PHASE_WAVES
#define DG_PHASE_WAVES 2  // min waves per SIMD of p1a, p3, dec_p3 (1 wave: above 256 VGPRs; 2: p3 554 -> 422 us)
#endif
#ifndef DG_EXP_WAVES
#define DG_EXP_WAVES (DG_EXP_LDS == 2 ? 4 : (DG_EXP_LDS ? 3 : 2))
#endif
#if DG_TU_HOT
DG_KERNEL void __launch_bounds__(128, DG_EXP_WAVES) k_exp_pm3d4(uint32_t n, const Fp* in, Fp* out) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
#if DG_EXP_LDS
  __shared__ uint32_t s_tab[DG_EXP_NTAB * 12 * 128];
  if (i >= n) return;
  fp_pow_pm3d4_lds(in[i], out[i], s_tab + threadIdx.x, 128u);
#else
  if (i >= n) return;
  out[i] = fp_pow_pm3d4_sos(in[i]);
#endif
}

DG_KERNEL void __launch_bounds__(128, DG_PHASE_WAVES) k_h2c_p1a(uint32_t R, const uint8_t* msgs, uint32_t msg_len, const uint8_t* dst,
                                                uint32_t dst_len, const XmdTail* xmd, H2cMap* st, Fp* nD) {
  uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= R) return;
  Fp2 u[2];
  if (msg_len == 32 && xmd)
    hash_to_field_xmd32(u, msgs + 32ull * r, xmd);
  else
    hash_to_field_fp2x2(u, msgs + (size_t)msg_len * r, msg_len, dst, dst_len);
  H2cMap s[2];
  h2c_p1a(u, s, nD[r]);
  st[2 * r].u = s[0].u;
  st[2 * r].x = s[0].x;
  st[2 * r + 1].u = s[1].u;
  st[2 * r + 1].x = s[1].x;
}
DG_KERNEL void __launch_bounds__(128) k_h2c_p1b(uint32_t R, H2cMap* st, const Fp* inv_nD, Fp* ein) {
  uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= R) return;
  H2cMap s[2] = {st[2 * r], st[2 * r + 1]};
  Fp e[2];
  h2c_p1b(s, inv_nD[r], e);
  st[2 * r] = s[0];
  st[2 * r + 1] = s[1];
  ein[2 * r] = e[0];
  ein[2 * r + 1] = e[1];
}
DG_KERNEL void __launch_bounds__(128) k_h2c_p2(uint32_t M, H2cMap* st, Fp* ein, const Fp* eout) {
  uint32_t m = blockIdx.x * blockDim.x + threadIdx.x;
  if (m >= M) return;
  H2cMap s = st[m];
  Fp c;
  h2c_p2(s, ein[m], eout[m], c);
  st[m].x = s.x;
  st[m].g = s.g;
  ein[m] = c;
}
DG_KERNEL void __launch_bounds__(128, DG_PHASE_WAVES) k_h2c_p3(uint32_t M, const H2cMap* st, const Fp* ein, const Fp* eout,
                                               G2JStore* iso) {
  uint32_t m = blockIdx.x * blockDim.x + threadIdx.x;
  if (m >= M) return;
  store_g2j(iso[m], h2c_p3(st[m], ein[m], eout[m]));
}
// P4: q0 + q1 and the norm of its Z (the value the batch inversion inverts), then the normalisation to
// Z = 1 with that inverse: the MSM and the scalar multiplications downstream use mixed additions
DG_KERNEL void __launch_bounds__(128) k_h2c_p4a(uint32_t R, const G2JStore* iso, G2JStore* outQ, Fp* nZ) {
  uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= R) return;
  G2J q = jac_add(load_g2j(iso[2 * r]), load_g2j(iso[2 * r + 1]));
  store_g2j(outQ[r], q);
  nZ[r] = fp2_norm(q.z);  // zero for the identity
}
DG_KERNEL void __launch_bounds__(128) k_h2c_p4b(uint32_t R, G2JStore* Q, const Fp* inv_nZ) {
  uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= R) return;
  G2J q = load_g2j(Q[r]);
  if (jac_is_inf(q)) return;  // stays the identity (Z = 0)
  Fp2 zinv{fp_mul(q.z.c0, inv_nZ[r]), fp_neg(fp_mul(q.z.c1, inv_nZ[r]))};  // fp2_inv(Z)
  store_g2j(Q[r], jac_from_aff(jac_to_aff_with_inv(q, zinv)));
}

// ---- batch inversion of n Fp values (Montgomery's trick over chunks of BINV_C consecutive values, a tree of
// chunk products, one safegcd at the root).  Zero inputs give zero.  Level arrays: vals (the inputs of the
// level), pre (their running products inside each chunk), up (one product per chunk = the next level's
// inputs); the inverses come back down: k_binv_down turns the inverse of each chunk product into the
// inverses of the chunk's values.
DG_KERNEL void __launch_bounds__(128) k_binv_up(uint32_t n, const Fp* vals, Fp* pre, Fp* up) {
  uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t a = j * BINV_C;
  if (a >= n) return;
  uint32_t b = a + BINV_C < n ? a + BINV_C : n;
  Fp acc = fp_one();
  for (uint32_t i = a; i < b; ++i) {
    Fp v = vals[i];
    acc = fp_mul(acc, fp_is_zero(v) ? fp_one() : v);
    pre[i] = acc;
  }
  up[j] = acc;
}
// inv: the inverses of the chunk products (the level above); out: the inverses of vals
DG_KERNEL void __launch_bounds__(128) k_binv_down(uint32_t n, const Fp* vals, const Fp* pre, const Fp* inv, Fp* out) {
  uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t a = j * BINV_C;
  if (a >= n) return;
  uint32_t b = a + BINV_C < n ? a + BINV_C : n;
  Fp I = inv[j];
  for (uint32_t i = b - 1; i > a; --i) {
    Fp v = vals[i];
    bool z = fp_is_zero(v);
    out[i] = z ? fp_zero() : fp_mul(I, pre[i - 1]);
    I = z ? I : fp_mul(I, v);
  }
  out[a] = fp_is_zero(vals[a]) ? fp_zero() : I;
}
// the top level (n <= BINV_C values), one lane: inverses of vals by one safegcd
DG_KERNEL void __launch_bounds__(64) k_binv_root(uint32_t n, const Fp* vals, Fp* out) {
  DG_HI();
  if (blockIdx.x * blockDim.x + threadIdx.x != 0) return;
  Fp pre[BINV_C];
  Fp acc = fp_one();
  for (uint32_t i = 0; i < n; ++i) {
    Fp v = vals[i];
    acc = fp_mul(acc, fp_is_zero(v) ? fp_one() : v);
    pre[i] = acc;
  }
  Fp I = fp_inv(acc);
  for (uint32_t i = n - 1; i > 0; --i) {
    Fp v = vals[i];
    bool z = fp_is_zero(v);
    out[i] = z ? fp_zero() : fp_mul(I, pre[i - 1]);
    I = z ? I : fp_mul(I, v);
  }
  out[0] = fp_is_zero(vals[0]) ? fp_zero() : I;
}

// ---- the same batch inversion as a block tree: a workgroup of BINV_T lanes takes BINV_T * BINV_K consecutive
// values (BINV_K per lane: running products in `pre`, the last one is the lane's leaf), multiplies the leaves up a
// binary tree in LDS and writes the root; the roots are inverted by the chunked form above (n / (BINV_T BINV_K) values); the
// down kernel rebuilds the tree, sends each node's inverse to its children (inv(left) = inv(node) * right) and
// walks each lane's values back.  Per value ~3 products, every lane busy: the chunked form left n / 32 lanes
// with 32 dependent products each (k_binv_down 113 us per 200k values, one pass per level).
__device__ __forceinline__ void binv_tree_up(Fp* T, uint32_t l) {
#pragma unroll 1
  for (uint32_t s = BINV_T / 2; s >= 1; s >>= 1) {
    __syncthreads();
    if (l < s) T[s + l] = fp_mul(T[2 * (s + l)], T[2 * (s + l) + 1]);
  }
  __syncthreads();
}
DG_KERNEL void __launch_bounds__(BINV_T) k_binv_blk_up(uint32_t n, const Fp* vals, Fp* pre, Fp* roots) {
  __shared__ Fp T[2 * BINV_T];
  const uint32_t l = threadIdx.x, a = (blockIdx.x * BINV_T + l) * BINV_K;
  Fp acc = fp_one();
  for (uint32_t c = 0; c < BINV_K && a + c < n; ++c) {
    const Fp v = vals[a + c];
    acc = fp_mul(acc, fp_is_zero(v) ? fp_one() : v);
    pre[a + c] = acc;
  }
  T[BINV_T + l] = acc;
  binv_tree_up(T, l);
  if (l == 0) roots[blockIdx.x] = T[1];
}
// rinv: the inverses of the block roots; out: the inverses of vals (zero for zero)
DG_KERNEL void __launch_bounds__(BINV_T) k_binv_blk_down(uint32_t n, const Fp* vals, const Fp* pre, const Fp* rinv,
                                                         Fp* out) {
  __shared__ Fp T[2 * BINV_T];
  const uint32_t l = threadIdx.x, a = (blockIdx.x * BINV_T + l) * BINV_K;
  const uint32_t b = a >= n ? a : (a + BINV_K < n ? a + BINV_K : n);  // this lane's values: [a, b)
  T[BINV_T + l] = b > a ? pre[b - 1] : fp_one();
  binv_tree_up(T, l);
  if (l == 0) T[1] = rinv[blockIdx.x];
#pragma unroll 1
  for (uint32_t s = 1; s < BINV_T; s <<= 1) {
    __syncthreads();
    if (l < s) {
      const uint32_t k = s + l;
      const Fp I = T[k], left = T[2 * k], right = T[2 * k + 1];
      T[2 * k] = fp_mul(I, right);
      T[2 * k + 1] = fp_mul(I, left);
    }
  }
  __syncthreads();
  if (b == a) return;
  Fp I = T[BINV_T + l];
  for (uint32_t i = b - 1; i > a; --i) {
    const Fp v = vals[i];
    const bool z = fp_is_zero(v);
    out[i] = z ? fp_zero() : fp_mul(I, pre[i - 1]);
    I = z ? I : fp_mul(I, v);
  }
  out[a] = fp_is_zero(vals[a]) ? fp_zero() : I;
}

// the roots of the block trees (n <= BINV_T * BINV_R values) inverted by one workgroup: running products of
// BINV_R values per lane, the LDS tree, one safegcd on lane 0, back down -- one launch instead of the chunked
// form's up / root / down chain
DG_KERNEL void __launch_bounds__(BINV_T) k_binv_blk_root(uint32_t n, const Fp* vals, Fp* out) {
  DG_HI();
  __shared__ Fp T[2 * BINV_T];
  const uint32_t l = threadIdx.x, a = l * BINV_R;
  // running products with compile-time indices (registers; a runtime-indexed array would live in scratch)
  Fp pre[BINV_R];
  Fp acc = fp_one();
#pragma unroll
  for (uint32_t c = 0; c < BINV_R; ++c) {
    const Fp v = a + c < n ? vals[a + c] : fp_one();
    acc = fp_mul(acc, fp_is_zero(v) ? fp_one() : v);
    pre[c] = acc;
  }
  T[BINV_T + l] = acc;
  binv_tree_up(T, l);
  if (l == 0) T[1] = fp_inv(T[1]);
#pragma unroll 1
  for (uint32_t s = 1; s < BINV_T; s <<= 1) {
    __syncthreads();
    if (l < s) {
      const uint32_t k = s + l;
      const Fp I = T[k], left = T[2 * k], right = T[2 * k + 1];
      T[2 * k] = fp_mul(I, right);
      T[2 * k + 1] = fp_mul(I, left);
    }
  }
  __syncthreads();
  Fp I = T[BINV_T + l];
#pragma unroll
  for (int c = BINV_R - 1; c >= 0; --c) {
    if (a + c >= n) continue;
    const Fp v = vals[a + c];
    const bool z = fp_is_zero(v);
    if (c > 0) {
      out[a + c] = z ? fp_zero() : fp_mul(I, pre[c - 1]);
      I = z ? I : fp_mul(I, v);
    } else {
      out[a] = z ? fp_zero() : I;
    }
  }
}

// decode of every item (96 B at sigs + stride*i + offset); items whose key did not decode are PK_DECODE
DG_KERNEL void __launch_bounds__(128) k_dec_p1(uint32_t n, const uint8_t* sigs, uint32_t stride, uint32_t offset,
                                               const uint32_t* item_slot, const uint8_t* key_status, DecState* ds,
                                               Fp* ein, uint8_t* status) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t slot = item_slot ? item_slot[i] : 0u;
  DecState d;
  Fp e;
  uint8_t st;
  if (key_status[slot] != DG_ST_OK_) {
    d.flags = 0;
    e = fp_zero();
    st = DG_ST_PK_DECODE_;
  } else {
    st = dec_p1(sigs + (size_t)stride * i + offset, d, e) ? DG_ST_SIG_DECODE_ : DG_ST_OK_;
  }
  ds[i] = d;
  ein[i] = e;
  status[i] = st;
}
DG_KERNEL void __launch_bounds__(128) k_dec_p2(uint32_t n, DecState* ds, Fp* ein, const Fp* eout, uint8_t* status) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  if (!(ds[i].flags & DEC_PENDING)) return;
  Fp c = fp_zero();
  if (!dec_p2(ds[i], ein[i], eout[i], c)) {
    ds[i].flags = 0;
    status[i] = DG_ST_SIG_DECODE_;
  }
  ein[i] = c;
}
// the sigma of item i into S, with the G2 subgroup check unless the batch checks subgroup membership on the
// MSM window sums (`subgroup` == 0, msm.h); claim the item's (round, slot) cell -- a taken cell, or a key
// outside the batch equation, sends the item to the individual check (`isolate`)
DG_KERNEL void __launch_bounds__(128, DG_PHASE_WAVES) k_dec_p3(uint32_t n, uint32_t k, uint32_t nslots, const uint32_t* item_slot,
                                               const DecState* ds, const Fp* ein, const Fp* eout, G2AStore* S,
                                               uint8_t* status, uint32_t* cell, uint8_t* isolate,
                                               uint32_t subgroup) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  isolate[i] = 0;
  const uint32_t flags = ds[i].flags;
  G2A a{fp2_zero(), fp2_zero(), true};
  bool ok = status[i] == DG_ST_OK_;
  if (ok && (flags & DEC_PENDING)) {
    ok = dec_p3(ds[i], ein[i], eout[i], subgroup != 0, a);
    if (!ok) {
      a = G2A{fp2_zero(), fp2_zero(), true};
      status[i] = DG_ST_SIG_DECODE_;
    }
  }
  store_g2a(S[i], a);
  if (ok) {
    const uint32_t slot = item_slot ? item_slot[i] : 0u;
    uint32_t old = slot < nslots ? atomicExch(&cell[(size_t)(i / k) * nslots + slot], 1u) : 1u;
    isolate[i] = old ? 1 : 0;
  }
}
#else
DG_KERNEL void __launch_bounds__(128, DG_EXP_WAVES) k_exp_pm3d4(uint32_t n, const Fp* in, Fp* out);
DG_KERNEL void __launch_bounds__(128, DG_PHASE_WAVES) k_h2c_p1a(uint32_t R, const uint8_t* msgs, uint32_t msg_len, const uint8_t* dst,
                                                uint32_t dst_len, const XmdTail* xmd, H2cMap* st, Fp* nD);
DG_KERNEL void __launch_bounds__(128) k_h2c_p1b(uint32_t R, H2cMap* st, const Fp* inv_nD, Fp* ein);
DG_KERNEL void __launch_bounds__(128) k_binv_up(uint32_t n, const Fp* vals, Fp* pre, Fp* up);
DG_KERNEL void __launch_bounds__(128) k_binv_down(uint32_t n, const Fp* vals, const Fp* pre, const Fp* inv, Fp* out);
DG_KERNEL void __launch_bounds__(64) k_binv_root(uint32_t n, const Fp* vals, Fp* out);
DG_KERNEL void __launch_bounds__(BINV_T) k_binv_blk_up(uint32_t n, const Fp* vals, Fp* pre, Fp* roots);
DG_KERNEL void __launch_bounds__(BINV_T) k_binv_blk_root(uint32_t n, const Fp* vals, Fp* out);
DG_KERNEL void __launch_bounds__(BINV_T) k_binv_blk_down(uint32_t n, const Fp* vals, const Fp* pre, const Fp* rinv,
                                                         Fp* out);
DG_KERNEL void __launch_bounds__(128) k_h2c_p2(uint32_t M, H2cMap* st, Fp* ein, const Fp* eout);
DG_KERNEL void __launch_bounds__(128, DG_PHASE_WAVES) k_h2c_p3(uint32_t M, const H2cMap* st, const Fp* ein, const Fp* eout,
                                               G2JStore* iso);
DG_KERNEL void __launch_bounds__(128) k_h2c_p4a(uint32_t R, const G2JStore* iso, G2JStore* outQ, Fp* nZ);
DG_KERNEL void __launch_bounds__(128) k_h2c_p4b(uint32_t R, G2JStore* Q, const Fp* inv_nZ);
DG_KERNEL void __launch_bounds__(128) k_dec_p1(uint32_t n, const uint8_t* sigs, uint32_t stride, uint32_t offset,
                                               const uint32_t* item_slot, const uint8_t* key_status, DecState* ds,
                                               Fp* ein, uint8_t* status);
DG_KERNEL void __launch_bounds__(128) k_dec_p2(uint32_t n, DecState* ds, Fp* ein, const Fp* eout, uint8_t* status);
DG_KERNEL void __launch_bounds__(128, DG_PHASE_WAVES) k_dec_p3(uint32_t n, uint32_t k, uint32_t nslots, const uint32_t* item_slot,
                                               const DecState* ds, const Fp* ein, const Fp* eout, G2AStore* S,
                                               uint8_t* status, uint32_t* cell, uint8_t* isolate,
                                               uint32_t subgroup);
#endif
#endif

}  // namespace dg
