/* CPU twin of the BLS12-381 threshold-BLS path -- TEST INFRASTRUCTURE ONLY.  See twin.h.
 *
 * Algorithms (all public, restated here; the reference's own copies live in the un-vendored
 * github.com/drand/bls12-381 v0.2.0 / github.com/drand/kyber modules, go.mod:9-10):
 *   - Montgomery CIOS over 6 x 64-bit limbs
 *   - Fp2 = Fp[u]/(u^2+1), Fp6 = Fp2[v]/(v^3-xi), Fp12 = Fp6[w]/(w^2-v), xi = 1+u
 *   - RFC 9380 hash_to_curve BLS12381G2_XMD:SHA-256_SSWU_RO_ (SSWU + 3-isogeny + h_eff via psi)
 *   - ZCash compressed encodings (G1 48 B, G2 96 B with x = c1 || c0)
 *   - optimal-ate Miller loop (homogeneous projective, M-type twist lines), final exponentiation
 *     with the hard part 3*Phi12(p)/r = (x-1)^2 (x+p)(x^2+p^2-1) + 3
 *   - tbls semantics of oracle/pyref/tbls.py
 */
#include "twin.h"

#include <pthread.h>
#include <stdlib.h>
#include <string.h>

typedef unsigned __int128 u128;
typedef uint64_t u64;
typedef struct { u64 l[6]; } fp;
typedef struct { fp c0, c1; } fp2;
typedef struct { fp2 c0, c1, c2; } fp6;
typedef struct { fp6 c0, c1; } fp12;
typedef struct { u64 l[4]; } fr;

static int g_count_on = 0;
static __thread u64 g_count = 0;
static u64 g_count_total = 0;
static pthread_mutex_t g_count_mu = PTHREAD_MUTEX_INITIALIZER;

/* ------------------------------------------------------------------------------------------ Fp */
static const fp P_MOD = {{0xb9feffffffffaaabULL, 0x1eabfffeb153ffffULL, 0x6730d2a0f6b0f624ULL, 0x64774b84f38512bfULL,
                          0x4b1ba7b6434bacd7ULL, 0x1a0111ea397fe69aULL}};
static u64 P_INV; /* -p^-1 mod 2^64 */
static fp FP_ONE, FP_R2;

static inline int fp_geq_p(const fp* a) {
  for (int i = 5; i >= 0; --i) {
    if (a->l[i] > P_MOD.l[i]) return 1;
    if (a->l[i] < P_MOD.l[i]) return 0;
  }
  return 1;
}
static inline void fp_sub_p(fp* a) {
  u64 br = 0;
  for (int i = 0; i < 6; ++i) {
    u128 d = (u128)a->l[i] - P_MOD.l[i] - br;
    a->l[i] = (u64)d;
    br = (u64)(d >> 64) & 1;
  }
}
static inline void fp_add(fp* r, const fp* a, const fp* b) {
  u64 c = 0;
  fp t;
  for (int i = 0; i < 6; ++i) {
    u128 s = (u128)a->l[i] + b->l[i] + c;
    t.l[i] = (u64)s;
    c = (u64)(s >> 64);
  }
  if (c || fp_geq_p(&t)) fp_sub_p(&t);
  *r = t;
}
static inline void fp_sub(fp* r, const fp* a, const fp* b) {
  u64 br = 0;
  fp t;
  for (int i = 0; i < 6; ++i) {
    u128 d = (u128)a->l[i] - b->l[i] - br;
    t.l[i] = (u64)d;
    br = (u64)(d >> 64) & 1;
  }
  if (br) {
    u64 c = 0;
    for (int i = 0; i < 6; ++i) {
      u128 s = (u128)t.l[i] + P_MOD.l[i] + c;
      t.l[i] = (u64)s;
      c = (u64)(s >> 64);
    }
  }
  *r = t;
}
static inline int fp_is_zero(const fp* a) {
  u64 o = 0;
  for (int i = 0; i < 6; ++i) o |= a->l[i];
  return o == 0;
}
static inline int fp_eq(const fp* a, const fp* b) { return memcmp(a, b, sizeof(fp)) == 0; }
static inline void fp_neg(fp* r, const fp* a) {
  if (fp_is_zero(a)) { *r = *a; return; }
  fp z;
  memset(&z, 0, sizeof z);
  fp_sub(r, &z, a);
}
static void fp_mul(fp* r, const fp* a, const fp* b) {
  if (g_count_on) g_count++;
  u64 t[8] = {0};
  for (int i = 0; i < 6; ++i) {
    u64 c = 0;
    for (int j = 0; j < 6; ++j) {
      u128 s = (u128)a->l[j] * b->l[i] + t[j] + c;
      t[j] = (u64)s;
      c = (u64)(s >> 64);
    }
    u128 s = (u128)t[6] + c;
    t[6] = (u64)s;
    t[7] = (u64)(s >> 64);
    u64 m = t[0] * P_INV;
    s = (u128)m * P_MOD.l[0] + t[0];
    c = (u64)(s >> 64);
    for (int j = 1; j < 6; ++j) {
      s = (u128)m * P_MOD.l[j] + t[j] + c;
      t[j - 1] = (u64)s;
      c = (u64)(s >> 64);
    }
    s = (u128)t[6] + c;
    t[5] = (u64)s;
    t[6] = t[7] + (u64)(s >> 64);
  }
  fp o;
  memcpy(o.l, t, 48);
  if (t[6] || fp_geq_p(&o)) fp_sub_p(&o);
  *r = o;
}
static inline void fp_sqr(fp* r, const fp* a) { fp_mul(r, a, a); }
static void fp_pow_u64s(fp* r, const fp* a, const u64* e, int nlimbs) {
  fp acc = FP_ONE;
  int started = 0;
  for (int i = nlimbs - 1; i >= 0; --i)
    for (int b = 63; b >= 0; --b) {
      if (started) fp_sqr(&acc, &acc);
      if ((e[i] >> b) & 1) {
        if (started) fp_mul(&acc, &acc, a);
        else { acc = *a; started = 1; }
      }
    }
  *r = acc;
}
static u64 E_PM2[6], E_PP1D4[6], E_PM1D2[6], E_PM3D4[6];
static void fp_inv(fp* r, const fp* a) { fp_pow_u64s(r, a, E_PM2, 6); }
static int fp_legendre_is_nonsquare(const fp* a) {
  if (fp_is_zero(a)) return 0;
  fp t;
  fp_pow_u64s(&t, a, E_PM1D2, 6);
  return !fp_eq(&t, &FP_ONE);
}
static int fp_sqrt(fp* r, const fp* a) {
  fp s, c;
  fp_pow_u64s(&s, a, E_PP1D4, 6);
  fp_sqr(&c, &s);
  if (!fp_eq(&c, a)) return 0;
  *r = s;
  return 1;
}
static void fp_from_int(fp* r, const u64 raw[6]) { fp t; memcpy(t.l, raw, 48); fp_mul(r, &t, &FP_R2); }
static void fp_to_int(u64 raw[6], const fp* a) {
  fp one;
  memset(&one, 0, sizeof one);
  one.l[0] = 1;
  fp t;
  fp_mul(&t, a, &one);
  memcpy(raw, t.l, 48);
}
static void fp_from_small(fp* r, u64 v) { u64 raw[6] = {v, 0, 0, 0, 0, 0}; fp_from_int(r, raw); }
/* big-endian 48 B -> raw limbs; returns 0 if >= p */
static int be48_to_raw(u64 raw[6], const uint8_t* b) {
  for (int i = 0; i < 6; ++i) {
    u64 v = 0;
    for (int k = 0; k < 8; ++k) v = (v << 8) | b[(5 - i) * 8 + k];
    raw[i] = v;
  }
  fp t;
  memcpy(t.l, raw, 48);
  return !fp_geq_p(&t);
}
static void raw_to_be48(uint8_t* b, const u64 raw[6]) {
  for (int i = 0; i < 6; ++i)
    for (int k = 0; k < 8; ++k) b[(5 - i) * 8 + k] = (uint8_t)(raw[i] >> (56 - 8 * k));
}
static void fp_to_be(uint8_t* b, const fp* a) { u64 raw[6]; fp_to_int(raw, a); raw_to_be48(b, raw); }
static int fp_from_be(fp* a, const uint8_t* b) {
  u64 raw[6];
  if (!be48_to_raw(raw, b)) return 0;
  fp_from_int(a, raw);
  return 1;
}
static int raw_gt_half(const u64 raw[6]) { /* raw > (p-1)/2 */
  u64 h[6];
  for (int i = 0; i < 6; ++i) h[i] = (P_MOD.l[i] >> 1) | (i < 5 ? (P_MOD.l[i + 1] << 63) : 0);
  for (int i = 5; i >= 0; --i) {
    if (raw[i] > h[i]) return 1;
    if (raw[i] < h[i]) return 0;
  }
  return 0;
}
static int fp_lex_largest(const fp* a) { u64 raw[6]; fp_to_int(raw, a); return raw_gt_half(raw); }

/* ------------------------------------------------------------------------------------------ Fp2 */
static inline void fp2_add(fp2* r, const fp2* a, const fp2* b) { fp_add(&r->c0, &a->c0, &b->c0); fp_add(&r->c1, &a->c1, &b->c1); }
static inline void fp2_sub(fp2* r, const fp2* a, const fp2* b) { fp_sub(&r->c0, &a->c0, &b->c0); fp_sub(&r->c1, &a->c1, &b->c1); }
static inline void fp2_neg(fp2* r, const fp2* a) { fp_neg(&r->c0, &a->c0); fp_neg(&r->c1, &a->c1); }
static inline void fp2_conj(fp2* r, const fp2* a) { r->c0 = a->c0; fp_neg(&r->c1, &a->c1); }
static inline int fp2_is_zero(const fp2* a) { return fp_is_zero(&a->c0) && fp_is_zero(&a->c1); }
static inline int fp2_eq(const fp2* a, const fp2* b) { return fp_eq(&a->c0, &b->c0) && fp_eq(&a->c1, &b->c1); }
static void fp2_mul(fp2* r, const fp2* a, const fp2* b) {
  fp t0, t1, t2, s0, s1;
  fp_mul(&t0, &a->c0, &b->c0);
  fp_mul(&t1, &a->c1, &b->c1);
  fp_add(&s0, &a->c0, &a->c1);
  fp_add(&s1, &b->c0, &b->c1);
  fp_mul(&t2, &s0, &s1);
  fp_sub(&r->c0, &t0, &t1);
  fp_sub(&t2, &t2, &t0);
  fp_sub(&r->c1, &t2, &t1);
}
static void fp2_sqr(fp2* r, const fp2* a) {
  fp s, d, m;
  fp_add(&s, &a->c0, &a->c1);
  fp_sub(&d, &a->c0, &a->c1);
  fp_mul(&m, &a->c0, &a->c1);
  fp_mul(&r->c0, &s, &d);
  fp_add(&r->c1, &m, &m);
}
static inline void fp2_mul_fp(fp2* r, const fp2* a, const fp* b) { fp_mul(&r->c0, &a->c0, b); fp_mul(&r->c1, &a->c1, b); }
static inline void fp2_mul_xi(fp2* r, const fp2* a) { /* (1+u) a */
  fp t0, t1;
  fp_sub(&t0, &a->c0, &a->c1);
  fp_add(&t1, &a->c0, &a->c1);
  r->c0 = t0;
  r->c1 = t1;
}
static void fp2_inv(fp2* r, const fp2* a) {
  fp n, t;
  fp_sqr(&n, &a->c0);
  fp_sqr(&t, &a->c1);
  fp_add(&n, &n, &t);
  fp_inv(&n, &n);
  fp_mul(&r->c0, &a->c0, &n);
  fp_mul(&t, &a->c1, &n);
  fp_neg(&r->c1, &t);
}
static void fp2_pow(fp2* r, const fp2* a, const u64* e, int nlimbs) {
  fp2 acc;
  int started = 0;
  for (int i = nlimbs - 1; i >= 0; --i)
    for (int b = 63; b >= 0; --b) {
      if (started) fp2_sqr(&acc, &acc);
      if ((e[i] >> b) & 1) {
        if (started) fp2_mul(&acc, &acc, a);
        else { acc = *a; started = 1; }
      }
    }
  if (!started) { acc.c0 = FP_ONE; memset(&acc.c1, 0, sizeof(fp)); }
  *r = acc;
}
static int fp2_is_square(const fp2* a) {
  fp n, t;
  fp_sqr(&n, &a->c0);
  fp_sqr(&t, &a->c1);
  fp_add(&n, &n, &t);
  return !fp_legendre_is_nonsquare(&n);
}
/* Adj & Rodriguez-Henriquez Alg. 9 */
static int fp2_sqrt(fp2* r, const fp2* a) {
  if (fp2_is_zero(a)) { *r = *a; return 1; }
  fp2 a1, alpha, a0, x0, t, minus_one;
  fp2_pow(&a1, a, E_PM3D4, 6);
  fp2_sqr(&alpha, &a1);
  fp2_mul(&alpha, &alpha, a);
  fp2_conj(&a0, &alpha); /* alpha^p */
  fp2_mul(&a0, &a0, &alpha);
  fp_neg(&minus_one.c0, &FP_ONE);
  memset(&minus_one.c1, 0, sizeof(fp));
  if (fp2_eq(&a0, &minus_one)) return 0;
  fp2_mul(&x0, &a1, a);
  if (fp2_eq(&alpha, &minus_one)) {
    /* x = u * x0 */
    fp2 u;
    memset(&u.c0, 0, sizeof(fp));
    u.c1 = FP_ONE;
    fp2_mul(&t, &u, &x0);
  } else {
    fp2 b, one;
    one.c0 = FP_ONE;
    memset(&one.c1, 0, sizeof(fp));
    fp2_add(&b, &one, &alpha);
    fp2_pow(&b, &b, E_PM1D2, 6);
    fp2_mul(&t, &b, &x0);
  }
  fp2 chk;
  fp2_sqr(&chk, &t);
  if (!fp2_eq(&chk, a)) return 0;
  *r = t;
  return 1;
}
static int fp2_sgn0(const fp2* a) {
  u64 r0[6], r1[6];
  fp_to_int(r0, &a->c0);
  fp_to_int(r1, &a->c1);
  int z0 = 1;
  for (int i = 0; i < 6; ++i) z0 &= r0[i] == 0;
  return (int)(r0[0] & 1) | (z0 & (int)(r1[0] & 1));
}
static int fp2_lex_largest(const fp2* a) {
  if (!fp_is_zero(&a->c1)) return fp_lex_largest(&a->c1);
  return fp_lex_largest(&a->c0);
}

/* ------------------------------------------------------------------------------------------ Fp6 / Fp12 */
static void fp6_add(fp6* r, const fp6* a, const fp6* b) { fp2_add(&r->c0, &a->c0, &b->c0); fp2_add(&r->c1, &a->c1, &b->c1); fp2_add(&r->c2, &a->c2, &b->c2); }
static void fp6_sub(fp6* r, const fp6* a, const fp6* b) { fp2_sub(&r->c0, &a->c0, &b->c0); fp2_sub(&r->c1, &a->c1, &b->c1); fp2_sub(&r->c2, &a->c2, &b->c2); }
static void fp6_neg(fp6* r, const fp6* a) { fp2_neg(&r->c0, &a->c0); fp2_neg(&r->c1, &a->c1); fp2_neg(&r->c2, &a->c2); }
static void fp6_mul(fp6* r, const fp6* a, const fp6* b) {
  fp2 v0, v1, v2, t0, t1, s, c0, c1, c2;
  fp2_mul(&v0, &a->c0, &b->c0);
  fp2_mul(&v1, &a->c1, &b->c1);
  fp2_mul(&v2, &a->c2, &b->c2);
  /* c0 = v0 + xi((a1+a2)(b1+b2) - v1 - v2) */
  fp2_add(&t0, &a->c1, &a->c2);
  fp2_add(&t1, &b->c1, &b->c2);
  fp2_mul(&s, &t0, &t1);
  fp2_sub(&s, &s, &v1);
  fp2_sub(&s, &s, &v2);
  fp2_mul_xi(&s, &s);
  fp2_add(&c0, &s, &v0);
  /* c1 = (a0+a1)(b0+b1) - v0 - v1 + xi v2 */
  fp2_add(&t0, &a->c0, &a->c1);
  fp2_add(&t1, &b->c0, &b->c1);
  fp2_mul(&s, &t0, &t1);
  fp2_sub(&s, &s, &v0);
  fp2_sub(&s, &s, &v1);
  fp2_mul_xi(&t0, &v2);
  fp2_add(&c1, &s, &t0);
  /* c2 = (a0+a2)(b0+b2) - v0 - v2 + v1 */
  fp2_add(&t0, &a->c0, &a->c2);
  fp2_add(&t1, &b->c0, &b->c2);
  fp2_mul(&s, &t0, &t1);
  fp2_sub(&s, &s, &v0);
  fp2_sub(&s, &s, &v2);
  fp2_add(&c2, &s, &v1);
  r->c0 = c0;
  r->c1 = c1;
  r->c2 = c2;
}
static void fp6_mul_v(fp6* r, const fp6* a) { /* v * (a0 + a1 v + a2 v^2) = xi a2 + a0 v + a1 v^2 */
  fp2 t;
  fp2_mul_xi(&t, &a->c2);
  r->c2 = a->c1;
  r->c1 = a->c0;
  r->c0 = t;
}
static void fp6_inv(fp6* r, const fp6* a) {
  fp2 c0, c1, c2, t, s;
  fp2_sqr(&c0, &a->c0);
  fp2_mul(&t, &a->c1, &a->c2);
  fp2_mul_xi(&t, &t);
  fp2_sub(&c0, &c0, &t);
  fp2_sqr(&c1, &a->c2);
  fp2_mul_xi(&c1, &c1);
  fp2_mul(&t, &a->c0, &a->c1);
  fp2_sub(&c1, &c1, &t);
  fp2_sqr(&c2, &a->c1);
  fp2_mul(&t, &a->c0, &a->c2);
  fp2_sub(&c2, &c2, &t);
  fp2_mul(&s, &a->c2, &c1);
  fp2_mul(&t, &a->c1, &c2);
  fp2_add(&s, &s, &t);
  fp2_mul_xi(&s, &s);
  fp2_mul(&t, &a->c0, &c0);
  fp2_add(&s, &s, &t);
  fp2_inv(&s, &s);
  fp2_mul(&r->c0, &c0, &s);
  fp2_mul(&r->c1, &c1, &s);
  fp2_mul(&r->c2, &c2, &s);
}
static void fp12_mul(fp12* r, const fp12* a, const fp12* b) {
  fp6 t0, t1, s0, s1, c1;
  fp6_mul(&t0, &a->c0, &b->c0);
  fp6_mul(&t1, &a->c1, &b->c1);
  fp6_add(&s0, &a->c0, &a->c1);
  fp6_add(&s1, &b->c0, &b->c1);
  fp6_mul(&c1, &s0, &s1);
  fp6_sub(&c1, &c1, &t0);
  fp6_sub(&c1, &c1, &t1);
  fp6_mul_v(&t1, &t1);
  fp6_add(&r->c0, &t0, &t1);
  r->c1 = c1;
}
static void fp12_sqr(fp12* r, const fp12* a) { fp12_mul(r, a, a); }
static void fp12_conj(fp12* r, const fp12* a) { r->c0 = a->c0; fp6_neg(&r->c1, &a->c1); }
static void fp12_inv(fp12* r, const fp12* a) {
  fp6 t0, t1;
  fp6_mul(&t0, &a->c0, &a->c0);
  fp6_mul(&t1, &a->c1, &a->c1);
  fp6_mul_v(&t1, &t1);
  fp6_sub(&t0, &t0, &t1);
  fp6_inv(&t0, &t0);
  fp6_mul(&r->c0, &a->c0, &t0);
  fp6_mul(&t1, &a->c1, &t0);
  fp6_neg(&r->c1, &t1);
}
static fp12 FP12_ONE;
static fp2 FROB6_G1, FROB6_G2, FROB12_D; /* xi^((p-1)/3), xi^(2(p-1)/3), xi^((p-1)/6) */
static void fp12_frob(fp12* r, const fp12* a) {
  fp12 t;
  fp2_conj(&t.c0.c0, &a->c0.c0);
  fp2_conj(&t.c0.c1, &a->c0.c1);
  fp2_mul(&t.c0.c1, &t.c0.c1, &FROB6_G1);
  fp2_conj(&t.c0.c2, &a->c0.c2);
  fp2_mul(&t.c0.c2, &t.c0.c2, &FROB6_G2);
  fp2_conj(&t.c1.c0, &a->c1.c0);
  fp2_conj(&t.c1.c1, &a->c1.c1);
  fp2_mul(&t.c1.c1, &t.c1.c1, &FROB6_G1);
  fp2_conj(&t.c1.c2, &a->c1.c2);
  fp2_mul(&t.c1.c2, &t.c1.c2, &FROB6_G2);
  fp2_mul(&t.c1.c0, &t.c1.c0, &FROB12_D);
  fp2_mul(&t.c1.c1, &t.c1.c1, &FROB12_D);
  fp2_mul(&t.c1.c2, &t.c1.c2, &FROB12_D);
  *r = t;
}
/* multiply by the sparse line c0 + c1 v + c4 v w  (slots 0, 1, 4) */
static void fp12_mul_014(fp12* f, const fp2* c0, const fp2* c1, const fp2* c4) {
  fp12 l;
  memset(&l, 0, sizeof l);
  l.c0.c0 = *c0;
  l.c0.c1 = *c1;
  l.c1.c1 = *c4;
  fp12_mul(f, f, &l);
}

/* ------------------------------------------------------------------------------------------ curves */
typedef struct { fp x, y, z; } g1j;    /* Jacobian, z = 0 is infinity */
typedef struct { fp2 x, y, z; } g2j;
static fp B1;
static fp2 B2;

static void g1_dbl(g1j* r, const g1j* p) {
  if (fp_is_zero(&p->z)) { *r = *p; return; }
  fp a, b, c, d, e, f, t;
  fp_sqr(&a, &p->x);
  fp_sqr(&b, &p->y);
  fp_sqr(&c, &b);
  fp_add(&t, &p->x, &b);
  fp_sqr(&d, &t);
  fp_sub(&d, &d, &a);
  fp_sub(&d, &d, &c);
  fp_add(&d, &d, &d);
  fp_add(&e, &a, &a);
  fp_add(&e, &e, &a);
  fp_sqr(&f, &e);
  g1j o;
  fp_sub(&o.x, &f, &d);
  fp_sub(&o.x, &o.x, &d);
  fp_mul(&o.z, &p->y, &p->z);
  fp_add(&o.z, &o.z, &o.z);
  fp_sub(&t, &d, &o.x);
  fp_mul(&o.y, &e, &t);
  fp_add(&c, &c, &c);
  fp_add(&c, &c, &c);
  fp_add(&c, &c, &c);
  fp_sub(&o.y, &o.y, &c);
  *r = o;
}
static void g1_add(g1j* r, const g1j* p, const g1j* q) {
  if (fp_is_zero(&p->z)) { *r = *q; return; }
  if (fp_is_zero(&q->z)) { *r = *p; return; }
  fp z1z1, z2z2, u1, u2, s1, s2, h, i, j, rr, v, t;
  fp_sqr(&z1z1, &p->z);
  fp_sqr(&z2z2, &q->z);
  fp_mul(&u1, &p->x, &z2z2);
  fp_mul(&u2, &q->x, &z1z1);
  fp_mul(&s1, &p->y, &q->z);
  fp_mul(&s1, &s1, &z2z2);
  fp_mul(&s2, &q->y, &p->z);
  fp_mul(&s2, &s2, &z1z1);
  if (fp_eq(&u1, &u2)) {
    if (fp_eq(&s1, &s2)) { g1_dbl(r, p); return; }
    memset(r, 0, sizeof *r);
    return;
  }
  fp_sub(&h, &u2, &u1);
  fp_add(&i, &h, &h);
  fp_sqr(&i, &i);
  fp_mul(&j, &h, &i);
  fp_sub(&rr, &s2, &s1);
  fp_add(&rr, &rr, &rr);
  fp_mul(&v, &u1, &i);
  g1j o;
  fp_sqr(&o.x, &rr);
  fp_sub(&o.x, &o.x, &j);
  fp_sub(&o.x, &o.x, &v);
  fp_sub(&o.x, &o.x, &v);
  fp_sub(&t, &v, &o.x);
  fp_mul(&o.y, &rr, &t);
  fp_mul(&t, &s1, &j);
  fp_add(&t, &t, &t);
  fp_sub(&o.y, &o.y, &t);
  fp_add(&t, &p->z, &q->z);
  fp_sqr(&t, &t);
  fp_sub(&t, &t, &z1z1);
  fp_sub(&t, &t, &z2z2);
  fp_mul(&o.z, &t, &h);
  *r = o;
}
static void g1_mul(g1j* r, const g1j* p, const u64* k, int nlimbs) {
  g1j acc;
  memset(&acc, 0, sizeof acc);
  for (int i = nlimbs - 1; i >= 0; --i)
    for (int b = 63; b >= 0; --b) {
      g1_dbl(&acc, &acc);
      if ((k[i] >> b) & 1) g1_add(&acc, &acc, p);
    }
  *r = acc;
}
static void g1_to_affine(fp* x, fp* y, const g1j* p) {
  fp zi, zi2;
  fp_inv(&zi, &p->z);
  fp_sqr(&zi2, &zi);
  fp_mul(x, &p->x, &zi2);
  fp_mul(&zi2, &zi2, &zi);
  fp_mul(y, &p->y, &zi2);
}

static void g2_dbl(g2j* r, const g2j* p) {
  if (fp2_is_zero(&p->z)) { *r = *p; return; }
  fp2 a, b, c, d, e, f, t;
  fp2_sqr(&a, &p->x);
  fp2_sqr(&b, &p->y);
  fp2_sqr(&c, &b);
  fp2_add(&t, &p->x, &b);
  fp2_sqr(&d, &t);
  fp2_sub(&d, &d, &a);
  fp2_sub(&d, &d, &c);
  fp2_add(&d, &d, &d);
  fp2_add(&e, &a, &a);
  fp2_add(&e, &e, &a);
  fp2_sqr(&f, &e);
  g2j o;
  fp2_sub(&o.x, &f, &d);
  fp2_sub(&o.x, &o.x, &d);
  fp2_mul(&o.z, &p->y, &p->z);
  fp2_add(&o.z, &o.z, &o.z);
  fp2_sub(&t, &d, &o.x);
  fp2_mul(&o.y, &e, &t);
  fp2_add(&c, &c, &c);
  fp2_add(&c, &c, &c);
  fp2_add(&c, &c, &c);
  fp2_sub(&o.y, &o.y, &c);
  *r = o;
}
static void g2_add(g2j* r, const g2j* p, const g2j* q) {
  if (fp2_is_zero(&p->z)) { *r = *q; return; }
  if (fp2_is_zero(&q->z)) { *r = *p; return; }
  fp2 z1z1, z2z2, u1, u2, s1, s2, h, i, j, rr, v, t;
  fp2_sqr(&z1z1, &p->z);
  fp2_sqr(&z2z2, &q->z);
  fp2_mul(&u1, &p->x, &z2z2);
  fp2_mul(&u2, &q->x, &z1z1);
  fp2_mul(&s1, &p->y, &q->z);
  fp2_mul(&s1, &s1, &z2z2);
  fp2_mul(&s2, &q->y, &p->z);
  fp2_mul(&s2, &s2, &z1z1);
  if (fp2_eq(&u1, &u2)) {
    if (fp2_eq(&s1, &s2)) { g2_dbl(r, p); return; }
    memset(r, 0, sizeof *r);
    return;
  }
  fp2_sub(&h, &u2, &u1);
  fp2_add(&i, &h, &h);
  fp2_sqr(&i, &i);
  fp2_mul(&j, &h, &i);
  fp2_sub(&rr, &s2, &s1);
  fp2_add(&rr, &rr, &rr);
  fp2_mul(&v, &u1, &i);
  g2j o;
  fp2_sqr(&o.x, &rr);
  fp2_sub(&o.x, &o.x, &j);
  fp2_sub(&o.x, &o.x, &v);
  fp2_sub(&o.x, &o.x, &v);
  fp2_sub(&t, &v, &o.x);
  fp2_mul(&o.y, &rr, &t);
  fp2_mul(&t, &s1, &j);
  fp2_add(&t, &t, &t);
  fp2_sub(&o.y, &o.y, &t);
  fp2_add(&t, &p->z, &q->z);
  fp2_sqr(&t, &t);
  fp2_sub(&t, &t, &z1z1);
  fp2_sub(&t, &t, &z2z2);
  fp2_mul(&o.z, &t, &h);
  *r = o;
}
static void g2_neg(g2j* r, const g2j* p) { r->x = p->x; fp2_neg(&r->y, &p->y); r->z = p->z; }
static void g2_mul(g2j* r, const g2j* p, const u64* k, int nlimbs) {
  g2j acc;
  memset(&acc, 0, sizeof acc);
  for (int i = nlimbs - 1; i >= 0; --i)
    for (int b = 63; b >= 0; --b) {
      g2_dbl(&acc, &acc);
      if ((k[i] >> b) & 1) g2_add(&acc, &acc, p);
    }
  *r = acc;
}
static const u64 Z_ABS = 0xd201000000010000ULL;
static void g2_mul_z(g2j* r, const g2j* p) { /* [z]P, z = -Z_ABS */
  g2j t;
  g2_mul(&t, p, &Z_ABS, 1);
  g2_neg(r, &t);
}
static fp2 PSI_CX, PSI_CY;
static void g2_psi(g2j* r, const g2j* p) {
  g2j o;
  fp2_conj(&o.x, &p->x);
  fp2_mul(&o.x, &o.x, &PSI_CX);
  fp2_conj(&o.y, &p->y);
  fp2_mul(&o.y, &o.y, &PSI_CY);
  fp2_conj(&o.z, &p->z);
  *r = o;
}
static int g2_eq(const g2j* p, const g2j* q) {
  int pz = fp2_is_zero(&p->z), qz = fp2_is_zero(&q->z);
  if (pz || qz) return pz && qz;
  fp2 z1z1, z2z2, a, b;
  fp2_sqr(&z1z1, &p->z);
  fp2_sqr(&z2z2, &q->z);
  fp2_mul(&a, &p->x, &z2z2);
  fp2_mul(&b, &q->x, &z1z1);
  if (!fp2_eq(&a, &b)) return 0;
  fp2_mul(&a, &p->y, &z2z2);
  fp2_mul(&a, &a, &q->z);
  fp2_mul(&b, &q->y, &z1z1);
  fp2_mul(&b, &b, &p->z);
  return fp2_eq(&a, &b);
}
static int g2_in_subgroup(const g2j* p) { /* psi(P) == [z]P */
  g2j a, b;
  g2_psi(&a, p);
  g2_mul_z(&b, p);
  return g2_eq(&a, &b);
}
static void g2_to_affine(fp2* x, fp2* y, const g2j* p) {
  fp2 zi, zi2;
  fp2_inv(&zi, &p->z);
  fp2_sqr(&zi2, &zi);
  fp2_mul(x, &p->x, &zi2);
  fp2_mul(&zi2, &zi2, &zi);
  fp2_mul(y, &p->y, &zi2);
}
static void g2_clear_cofactor(g2j* r, const g2j* p) { /* RFC 9380 App. G.3 */
  g2j t1, t2, t3;
  g2_mul_z(&t1, p);
  g2_psi(&t2, p);
  g2_dbl(&t3, p);
  g2_psi(&t3, &t3);
  g2_psi(&t3, &t3);
  g2j nt2;
  g2_neg(&nt2, &t2);
  g2_add(&t3, &t3, &nt2);
  g2_add(&t2, &t1, &t2);
  g2_mul_z(&t2, &t2);
  g2_add(&t3, &t3, &t2);
  g2j n;
  g2_neg(&n, &t1);
  g2_add(&t3, &t3, &n);
  g2_neg(&n, p);
  g2_add(r, &t3, &n);
}

/* ------------------------------------------------------------------------------------------ encodings */
static void g1_compress(uint8_t out[48], const g1j* p) {
  if (fp_is_zero(&p->z)) { memset(out, 0, 48); out[0] = 0xc0; return; }
  fp x, y;
  g1_to_affine(&x, &y, p);
  fp_to_be(out, &x);
  out[0] |= 0x80;
  if (fp_lex_largest(&y)) out[0] |= 0x20;
}
static const u64 R_ORD[4] = {0xffffffff00000001ULL, 0x53bda402fffe5bfeULL, 0x3339d80809a1d805ULL, 0x73eda753299d7d48ULL};
static int g1_decompress(g1j* p, const uint8_t in[48]) {
  uint8_t f = in[0];
  if (!(f & 0x80)) return 0;
  if (f & 0x40) {
    if (f != 0xc0) return 0;
    for (int i = 1; i < 48; ++i) if (in[i]) return 0;
    memset(p, 0, sizeof *p);
    return 1;
  }
  uint8_t b[48];
  memcpy(b, in, 48);
  b[0] &= 0x1f;
  fp x, y, t;
  if (!fp_from_be(&x, b)) return 0;
  fp_sqr(&t, &x);
  fp_mul(&t, &t, &x);
  fp_add(&t, &t, &B1);
  if (!fp_sqrt(&y, &t)) return 0;
  if (((f & 0x20) != 0) != fp_lex_largest(&y)) fp_neg(&y, &y);
  p->x = x;
  p->y = y;
  p->z = FP_ONE;
  g1j c;
  g1_mul(&c, p, R_ORD, 4);
  if (!fp_is_zero(&c.z)) return 0;
  return 1;
}
static void g2_compress(uint8_t out[96], const g2j* p) {
  if (fp2_is_zero(&p->z)) { memset(out, 0, 96); out[0] = 0xc0; return; }
  fp2 x, y;
  g2_to_affine(&x, &y, p);
  fp_to_be(out, &x.c1);
  fp_to_be(out + 48, &x.c0);
  out[0] |= 0x80;
  if (fp2_lex_largest(&y)) out[0] |= 0x20;
}
static int g2_decompress(g2j* p, const uint8_t in[96]) {
  uint8_t f = in[0];
  if (!(f & 0x80)) return 0;
  if (f & 0x40) {
    if (f != 0xc0) return 0;
    for (int i = 1; i < 96; ++i) if (in[i]) return 0;
    memset(p, 0, sizeof *p);
    return 1;
  }
  uint8_t b[48];
  memcpy(b, in, 48);
  b[0] &= 0x1f;
  fp2 x, y, t;
  if (!fp_from_be(&x.c1, b)) return 0;
  if (!fp_from_be(&x.c0, in + 48)) return 0;
  fp2_sqr(&t, &x);
  fp2_mul(&t, &t, &x);
  fp2_add(&t, &t, &B2);
  if (!fp2_sqrt(&y, &t)) return 0;
  if (((f & 0x20) != 0) != fp2_lex_largest(&y)) fp2_neg(&y, &y);
  p->x = x;
  p->y = y;
  p->z.c0 = FP_ONE;
  memset(&p->z.c1, 0, sizeof(fp));
  if (!g2_in_subgroup(p)) return 0;
  return 1;
}

/* ------------------------------------------------------------------------------------------ SHA-256 */
typedef struct { uint32_t h[8]; uint8_t buf[64]; size_t len; u64 total; } sha256_ctx;
static const uint32_t K256[64] = {
    0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5, 0xd807aa98, 0x12835b01,
    0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174, 0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc,
    0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da, 0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147,
    0x06ca6351, 0x14292967, 0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
    0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070, 0x19a4c116, 0x1e376c08,
    0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3, 0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208,
    0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2};
#define ROR(x, n) (((x) >> (n)) | ((x) << (32 - (n))))
static void sha256_block(uint32_t h[8], const uint8_t* p) {
  uint32_t w[64];
  for (int i = 0; i < 16; ++i) w[i] = (uint32_t)p[4 * i] << 24 | (uint32_t)p[4 * i + 1] << 16 | (uint32_t)p[4 * i + 2] << 8 | p[4 * i + 3];
  for (int i = 16; i < 64; ++i) {
    uint32_t s0 = ROR(w[i - 15], 7) ^ ROR(w[i - 15], 18) ^ (w[i - 15] >> 3);
    uint32_t s1 = ROR(w[i - 2], 17) ^ ROR(w[i - 2], 19) ^ (w[i - 2] >> 10);
    w[i] = w[i - 16] + s0 + w[i - 7] + s1;
  }
  uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], hh = h[7];
  for (int i = 0; i < 64; ++i) {
    uint32_t t1 = hh + (ROR(e, 6) ^ ROR(e, 11) ^ ROR(e, 25)) + ((e & f) ^ (~e & g)) + K256[i] + w[i];
    uint32_t t2 = (ROR(a, 2) ^ ROR(a, 13) ^ ROR(a, 22)) + ((a & b) ^ (a & c) ^ (b & c));
    hh = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
  }
  h[0] += a; h[1] += b; h[2] += c; h[3] += d; h[4] += e; h[5] += f; h[6] += g; h[7] += hh;
}
static void sha256_init(sha256_ctx* c) {
  static const uint32_t iv[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a, 0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
  memcpy(c->h, iv, 32);
  c->len = 0;
  c->total = 0;
}
static void sha256_update(sha256_ctx* c, const uint8_t* d, size_t n) {
  c->total += n;
  while (n) {
    size_t k = 64 - c->len;
    if (k > n) k = n;
    memcpy(c->buf + c->len, d, k);
    c->len += k;
    d += k;
    n -= k;
    if (c->len == 64) { sha256_block(c->h, c->buf); c->len = 0; }
  }
}
static void sha256_final(sha256_ctx* c, uint8_t out[32]) {
  u64 bits = c->total * 8;
  uint8_t pad = 0x80;
  sha256_update(c, &pad, 1);
  uint8_t z = 0;
  while (c->len != 56) sha256_update(c, &z, 1);
  uint8_t lb[8];
  for (int i = 0; i < 8; ++i) lb[i] = (uint8_t)(bits >> (56 - 8 * i));
  sha256_update(c, lb, 8);
  for (int i = 0; i < 8; ++i) {
    out[4 * i] = (uint8_t)(c->h[i] >> 24); out[4 * i + 1] = (uint8_t)(c->h[i] >> 16);
    out[4 * i + 2] = (uint8_t)(c->h[i] >> 8); out[4 * i + 3] = (uint8_t)c->h[i];
  }
}

/* ------------------------------------------------------------------------------------------ hash to G2 */
static void expand_message_xmd(uint8_t* out, size_t len, const uint8_t* msg, size_t msg_len, const uint8_t* dst,
                               size_t dst_len) {
  size_t ell = (len + 31) / 32;
  uint8_t b0[32], bi[32], z[64] = {0}, lib[2] = {(uint8_t)(len >> 8), (uint8_t)len}, zero = 0, dl = (uint8_t)dst_len;
  sha256_ctx c;
  sha256_init(&c);
  sha256_update(&c, z, 64);
  sha256_update(&c, msg, msg_len);
  sha256_update(&c, lib, 2);
  sha256_update(&c, &zero, 1);
  sha256_update(&c, dst, dst_len);
  sha256_update(&c, &dl, 1);
  sha256_final(&c, b0);
  uint8_t one = 1;
  sha256_init(&c);
  sha256_update(&c, b0, 32);
  sha256_update(&c, &one, 1);
  sha256_update(&c, dst, dst_len);
  sha256_update(&c, &dl, 1);
  sha256_final(&c, bi);
  memcpy(out, bi, len < 32 ? len : 32);
  for (size_t i = 2; i <= ell; ++i) {
    uint8_t x[32], ib = (uint8_t)i;
    for (int k = 0; k < 32; ++k) x[k] = b0[k] ^ bi[k];
    sha256_init(&c);
    sha256_update(&c, x, 32);
    sha256_update(&c, &ib, 1);
    sha256_update(&c, dst, dst_len);
    sha256_update(&c, &dl, 1);
    sha256_final(&c, bi);
    size_t off = (i - 1) * 32, k = len - off < 32 ? len - off : 32;
    memcpy(out + off, bi, k);
  }
}
/* 64 B big-endian -> Fp (mod p), via hi*2^256 + lo with R^2 / R^3 scaling */
static fp FP_2_256;
static void fp_from_be64(fp* r, const uint8_t* b) {
  /* value = hi(32 B) * 2^256 + lo(32 B) */
  u64 hi[6] = {0}, lo[6] = {0};
  for (int i = 0; i < 4; ++i) {
    u64 vh = 0, vl = 0;
    for (int k = 0; k < 8; ++k) { vh = (vh << 8) | b[(3 - i) * 8 + k]; vl = (vl << 8) | b[32 + (3 - i) * 8 + k]; }
    hi[i] = vh;
    lo[i] = vl;
  }
  fp h, l;
  fp_from_int(&h, hi);
  fp_from_int(&l, lo);
  fp_mul(&h, &h, &FP_2_256);
  fp_add(r, &h, &l);
}
static fp2 SSWU_A, SSWU_B, SSWU_Z, ISO_XNUM[4], ISO_XDEN[3], ISO_YNUM[4], ISO_YDEN[4];
static void map_to_curve_sswu(fp2* ox, fp2* oy, const fp2* u) {
  fp2 zu2, den, x1, gx1, x, y, t, one;
  one.c0 = FP_ONE;
  memset(&one.c1, 0, sizeof(fp));
  fp2_sqr(&t, u);
  fp2_mul(&zu2, &SSWU_Z, &t);
  fp2_sqr(&den, &zu2);
  fp2_add(&den, &den, &zu2);
  if (fp2_is_zero(&den)) {
    fp2_mul(&t, &SSWU_Z, &SSWU_A);
    fp2_inv(&t, &t);
    fp2_mul(&x1, &SSWU_B, &t);
  } else {
    fp2_inv(&t, &den);
    fp2_add(&t, &t, &one);
    fp2 nb, ia;
    fp2_neg(&nb, &SSWU_B);
    fp2_inv(&ia, &SSWU_A);
    fp2_mul(&nb, &nb, &ia);
    fp2_mul(&x1, &nb, &t);
  }
  fp2_sqr(&gx1, &x1);
  fp2_add(&gx1, &gx1, &SSWU_A);
  fp2_mul(&gx1, &gx1, &x1);
  fp2_add(&gx1, &gx1, &SSWU_B);
  if (fp2_is_square(&gx1)) {
    x = x1;
    fp2_sqrt(&y, &gx1);
  } else {
    fp2 gx2;
    fp2_mul(&x, &zu2, &x1);
    fp2_sqr(&gx2, &x);
    fp2_add(&gx2, &gx2, &SSWU_A);
    fp2_mul(&gx2, &gx2, &x);
    fp2_add(&gx2, &gx2, &SSWU_B);
    fp2_sqrt(&y, &gx2);
  }
  if (fp2_sgn0(u) != fp2_sgn0(&y)) fp2_neg(&y, &y);
  *ox = x;
  *oy = y;
}
static void poly_eval(fp2* r, const fp2* c, int n, const fp2* x) {
  fp2 acc = c[n - 1];
  for (int i = n - 2; i >= 0; --i) {
    fp2_mul(&acc, &acc, x);
    fp2_add(&acc, &acc, &c[i]);
  }
  *r = acc;
}
static void iso_map(g2j* r, const fp2* x, const fp2* y) {
  fp2 xn, xd, yn, yd;
  poly_eval(&xn, ISO_XNUM, 4, x);
  poly_eval(&xd, ISO_XDEN, 3, x);
  poly_eval(&yn, ISO_YNUM, 4, x);
  poly_eval(&yd, ISO_YDEN, 4, x);
  if (fp2_is_zero(&xd) || fp2_is_zero(&yd)) { memset(r, 0, sizeof *r); return; }
  /* Jacobian: X = xn*xd*yd^2 ... use Z = xd*yd: x = X/Z^2, y = Y/Z^3 */
  fp2 z, z2, t;
  fp2_mul(&z, &xd, &yd);
  fp2_sqr(&z2, &z);
  /* X = xn/xd * Z^2 = xn * xd * yd^2 */
  fp2_sqr(&t, &yd);
  fp2_mul(&t, &t, &xd);
  fp2_mul(&r->x, &xn, &t);
  /* Y = y*yn/yd * Z^3 = y * yn * xd^3 * yd^2 */
  fp2_mul(&t, &z2, &xd); /* xd^3 yd^2 */
  fp2_mul(&t, &t, &yn);
  fp2_mul(&r->y, &t, y);
  r->z = z;
}
static void hash_to_g2_point(g2j* out, const uint8_t* msg, size_t msg_len, const uint8_t* dst, size_t dst_len) {
  uint8_t ub[256];
  expand_message_xmd(ub, 256, msg, msg_len, dst, dst_len);
  fp2 u[2];
  for (int i = 0; i < 2; ++i) {
    fp_from_be64(&u[i].c0, ub + 128 * i);
    fp_from_be64(&u[i].c1, ub + 128 * i + 64);
  }
  g2j q[2];
  for (int i = 0; i < 2; ++i) {
    fp2 x, y;
    map_to_curve_sswu(&x, &y, &u[i]);
    iso_map(&q[i], &x, &y);
  }
  g2j s;
  g2_add(&s, &q[0], &q[1]);
  g2_clear_cofactor(out, &s);
}
static const uint8_t DST_NUL[] = "BLS_SIG_BLS12381G2_XMD:SHA-256_SSWU_RO_NUL_";
#define DST_NUL_LEN 43
/* the hash-to-G2 DST of sign / verify (the one unpinned parameter of the suite):
 * NUL by default, switchable with twin_set_dst like the library's dg_set_hash_dst */
static uint8_t g_dst[255];
static size_t g_dst_len = 0;
static const uint8_t* cur_dst(size_t* len) {
  if (g_dst_len == 0) {
    *len = DST_NUL_LEN;
    return DST_NUL;
  }
  *len = g_dst_len;
  return g_dst;
}

/* ------------------------------------------------------------------------------------------ pairing */
typedef struct { fp2 x, y, z; } g2p; /* homogeneous projective */
static fp2 B2_3; /* 3 b' */
static fp TWO_INV;
static void line_dbl(g2p* T, fp2* c0, fp2* c1, fp2* c4, const fp* px, const fp* py) {
  fp2 a, b, c, e, f, g, h, j, t;
  fp2_mul(&a, &T->x, &T->y);
  fp2_mul_fp(&a, &a, &TWO_INV);
  fp2_sqr(&b, &T->y);
  fp2_sqr(&c, &T->z);
  fp2_mul(&e, &B2_3, &c);
  fp2_add(&f, &e, &e);
  fp2_add(&f, &f, &e);
  fp2_add(&g, &b, &f);
  fp2_mul_fp(&g, &g, &TWO_INV);
  fp2_add(&t, &T->y, &T->z);
  fp2_sqr(&h, &t);
  fp2_sub(&h, &h, &b);
  fp2_sub(&h, &h, &c);
  fp2_sqr(&j, &T->x);
  /* line: (e - b) + 3X^2 xP v - h yP vw  (overall sign irrelevant) */
  fp2_sub(c0, &e, &b);
  fp2_add(&t, &j, &j);
  fp2_add(&t, &t, &j);
  fp2_mul_fp(c1, &t, px);
  fp2_neg(&t, &h);
  fp2_mul_fp(c4, &t, py);
  fp2 nx, ny, nz, e2;
  fp2_sub(&t, &b, &f);
  fp2_mul(&nx, &a, &t);
  fp2_sqr(&e2, &e);
  fp2_sqr(&ny, &g);
  fp2_sub(&ny, &ny, &e2);
  fp2_sub(&ny, &ny, &e2);
  fp2_sub(&ny, &ny, &e2);
  fp2_mul(&nz, &b, &h);
  T->x = nx;
  T->y = ny;
  T->z = nz;
}
static void line_add(g2p* T, const fp2* qx, const fp2* qy, fp2* c0, fp2* c1, fp2* c4, const fp* px, const fp* py) {
  fp2 theta, lambda, c, d, e, f, g, h, t;
  fp2_mul(&t, qy, &T->z);
  fp2_sub(&theta, &T->y, &t);
  fp2_mul(&t, qx, &T->z);
  fp2_sub(&lambda, &T->x, &t);
  fp2_sqr(&c, &theta);
  fp2_sqr(&d, &lambda);
  fp2_mul(&e, &lambda, &d);
  fp2_mul(&f, &T->z, &c);
  fp2_mul(&g, &T->x, &d);
  fp2_add(&h, &e, &f);
  fp2_sub(&h, &h, &g);
  fp2_sub(&h, &h, &g);
  fp2 nx, ny, nz;
  fp2_mul(&nx, &lambda, &h);
  fp2_sub(&t, &g, &h);
  fp2_mul(&ny, &theta, &t);
  fp2_mul(&t, &e, &T->y);
  fp2_sub(&ny, &ny, &t);
  fp2_mul(&nz, &T->z, &e);
  T->x = nx;
  T->y = ny;
  T->z = nz;
  /* line: (theta xQ - lambda yQ) - theta xP v + lambda yP vw */
  fp2 j2;
  fp2_mul(&j2, &theta, qx);
  fp2_mul(&t, &lambda, qy);
  fp2_sub(c0, &j2, &t);
  fp2_neg(&t, &theta);
  fp2_mul_fp(c1, &t, px);
  fp2_mul_fp(c4, &lambda, py);
}
/* pairs with infinity on either side contribute 1 */
static void miller_loop_multi(fp12* f, int npairs, const fp* px, const fp* py, const fp2* qx, const fp2* qy) {
  g2p T[4];
  *f = FP12_ONE;
  for (int k = 0; k < npairs; ++k) {
    T[k].x = qx[k];
    T[k].y = qy[k];
    T[k].z.c0 = FP_ONE;
    memset(&T[k].z.c1, 0, sizeof(fp));
  }
  for (int b = 62; b >= 0; --b) {
    fp12_sqr(f, f);
    for (int k = 0; k < npairs; ++k) {
      fp2 c0, c1, c4;
      line_dbl(&T[k], &c0, &c1, &c4, &px[k], &py[k]);
      fp12_mul_014(f, &c0, &c1, &c4);
    }
    if ((Z_ABS >> b) & 1)
      for (int k = 0; k < npairs; ++k) {
        fp2 c0, c1, c4;
        line_add(&T[k], &qx[k], &qy[k], &c0, &c1, &c4, &px[k], &py[k]);
        fp12_mul_014(f, &c0, &c1, &c4);
      }
  }
  fp12_conj(f, f);
}
static void cyc_exp_z(fp12* r, const fp12* a) { /* a^z, z negative, a in cyclotomic subgroup */
  fp12 acc = *a;
  for (int b = 62; b >= 0; --b) {
    fp12_sqr(&acc, &acc);
    if ((Z_ABS >> b) & 1) fp12_mul(&acc, &acc, a);
  }
  fp12_conj(r, &acc);
}
static void final_exp(fp12* r, const fp12* f) {
  fp12 t, f1, f2, t0, t1, a, b, c;
  fp12_conj(&t, f);
  fp12_inv(&f1, f);
  fp12_mul(&f1, &t, &f1);       /* f^(p^6-1) */
  fp12_frob(&t, &f1);
  fp12_frob(&t, &t);
  fp12_mul(&f2, &t, &f1);       /* ^(p^2+1) */
  cyc_exp_z(&t0, &f2);
  fp12_conj(&t, &f2);
  fp12_mul(&t0, &t0, &t);       /* f2^(z-1) */
  cyc_exp_z(&t1, &t0);
  fp12_conj(&t, &t0);
  fp12_mul(&t1, &t1, &t);       /* f2^((z-1)^2) */
  cyc_exp_z(&a, &t1);
  fp12_frob(&t, &t1);
  fp12_mul(&a, &a, &t);         /* ^(z+p) */
  cyc_exp_z(&b, &a);
  cyc_exp_z(&b, &b);
  fp12_frob(&t, &a);
  fp12_frob(&t, &t);
  fp12_mul(&b, &b, &t);
  fp12_conj(&t, &a);
  fp12_mul(&b, &b, &t);         /* ^(z^2+p^2-1) */
  fp12_sqr(&c, &f2);
  fp12_mul(&c, &c, &f2);
  fp12_mul(r, &b, &c);
}
static int fp12_is_one(const fp12* a) { return memcmp(a, &FP12_ONE, sizeof(fp12)) == 0; }

/* ------------------------------------------------------------------------------------------ init */
static int g_inited = 0;
static pthread_once_t g_once = PTHREAD_ONCE_INIT;
static void fp_from_hex(fp* r, const char* hex) {
  u64 raw[6] = {0};
  size_t n = strlen(hex);
  for (size_t i = 0; i < n; ++i) {
    char ch = hex[n - 1 - i];
    u64 v = (ch >= '0' && ch <= '9') ? (u64)(ch - '0') : (u64)((ch | 32) - 'a' + 10);
    raw[i / 16] |= v << (4 * (i % 16));
  }
  fp_from_int(r, raw);
}
static void fp2_from_hex(fp2* r, const char* a, const char* b) { fp_from_hex(&r->c0, a); fp_from_hex(&r->c1, b); }
static void sub_small(u64* e, u64 v) { /* e -= v */
  for (int i = 0; i < 6; ++i) {
    u64 o = e[i];
    e[i] -= v;
    v = o < v;
    if (!v) break;
  }
}
static void shr(u64* e, int k) {
  for (int i = 0; i < 6; ++i) e[i] = (e[i] >> k) | (i < 5 ? e[i + 1] << (64 - k) : 0);
}
static void do_init(void) {
  /* -p^-1 mod 2^64 */
  u64 inv = 1;
  for (int i = 0; i < 7; ++i) inv *= 2 - P_MOD.l[0] * inv;
  P_INV = (u64)0 - inv;
  /* R mod p and R^2 mod p by doubling */
  fp x;
  memset(&x, 0, sizeof x);
  x.l[0] = 1;
  for (int i = 0; i < 384; ++i) fp_add(&x, &x, &x);
  FP_ONE = x;
  for (int i = 0; i < 384; ++i) fp_add(&x, &x, &x);
  FP_R2 = x;
  memcpy(E_PM2, P_MOD.l, 48); sub_small(E_PM2, 2);
  memcpy(E_PP1D4, P_MOD.l, 48); /* (p+1)/4 = (p-3)/4 + 1 */
  sub_small(E_PP1D4, 3); shr(E_PP1D4, 2);
  memcpy(E_PM3D4, E_PP1D4, 48);
  { u64 c = 1; for (int i = 0; i < 6 && c; ++i) { E_PP1D4[i] += c; c = E_PP1D4[i] == 0; } }
  memcpy(E_PM1D2, P_MOD.l, 48); sub_small(E_PM1D2, 1); shr(E_PM1D2, 1);
  fp_from_small(&B1, 4);
  fp_from_small(&B2.c0, 4);
  fp_from_small(&B2.c1, 4);
  fp2_add(&B2_3, &B2, &B2);
  fp2_add(&B2_3, &B2_3, &B2);
  fp two;
  fp_from_small(&two, 2);
  fp_inv(&TWO_INV, &two);
  { u64 raw[6] = {0}; raw[4] = 1; fp_from_int(&FP_2_256, raw); }
  memset(&FP12_ONE, 0, sizeof FP12_ONE);
  FP12_ONE.c0.c0.c0 = FP_ONE;
  /* frobenius constants */
  fp2 xi;
  xi.c0 = FP_ONE;
  xi.c1 = FP_ONE;
  u64 e[6];
  memcpy(e, P_MOD.l, 48); sub_small(e, 1);
  u64 e3[6], e6[6], e2[6];
  /* (p-1)/3, (p-1)/6, (p-1)/2 via division of 6-limb number by small */
  for (int d = 0; d < 3; ++d) {
    u64 div = d == 0 ? 3 : (d == 1 ? 6 : 2);
    u64* out = d == 0 ? e3 : (d == 1 ? e6 : e2);
    u128 rem = 0;
    for (int i = 5; i >= 0; --i) {
      u128 cur = (rem << 64) | e[i];
      out[i] = (u64)(cur / div);
      rem = cur % div;
    }
  }
  fp2_pow(&FROB6_G1, &xi, e3, 6);
  fp2_sqr(&FROB6_G2, &FROB6_G1);
  fp2_pow(&FROB12_D, &xi, e6, 6);
  fp2_inv(&PSI_CX, &FROB6_G1);
  fp2 t;
  fp2_pow(&t, &xi, e2, 6);
  fp2_inv(&PSI_CY, &t);
  /* SSWU / isogeny constants (RFC 9380 §8.8.2, App. E.3) */
  fp zero;
  memset(&zero, 0, sizeof zero);
  fp_from_small(&SSWU_A.c1, 240); SSWU_A.c0 = zero;
  fp_from_small(&SSWU_B.c0, 1012); SSWU_B.c1 = SSWU_B.c0;
  fp_from_small(&SSWU_Z.c0, 2); fp_neg(&SSWU_Z.c0, &SSWU_Z.c0);
  fp_from_small(&SSWU_Z.c1, 1); fp_neg(&SSWU_Z.c1, &SSWU_Z.c1);
  fp2_from_hex(&ISO_XNUM[0], "5c759507e8e333ebb5b7a9a47d7ed8532c52d39fd3a042a88b58423c50ae15d5c2638e343d9c71c6238aaaaaaaa97d6",
               "5c759507e8e333ebb5b7a9a47d7ed8532c52d39fd3a042a88b58423c50ae15d5c2638e343d9c71c6238aaaaaaaa97d6");
  fp2_from_hex(&ISO_XNUM[1], "0", "11560bf17baa99bc32126fced787c88f984f87adf7ae0c7f9a208c6b4f20a4181472aaa9cb8d555526a9ffffffffc71a");
  fp2_from_hex(&ISO_XNUM[2], "11560bf17baa99bc32126fced787c88f984f87adf7ae0c7f9a208c6b4f20a4181472aaa9cb8d555526a9ffffffffc71e",
               "8ab05f8bdd54cde190937e76bc3e447cc27c3d6fbd7063fcd104635a790520c0a395554e5c6aaaa9354ffffffffe38d");
  fp2_from_hex(&ISO_XNUM[3], "171d6541fa38ccfaed6dea691f5fb614cb14b4e7f4e810aa22d6108f142b85757098e38d0f671c7188e2aaaaaaaa5ed1", "0");
  fp2_from_hex(&ISO_XDEN[0], "0", "1a0111ea397fe69a4b1ba7b6434bacd764774b84f38512bf6730d2a0f6b0f6241eabfffeb153ffffb9feffffffffaa63");
  fp2_from_hex(&ISO_XDEN[1], "c", "1a0111ea397fe69a4b1ba7b6434bacd764774b84f38512bf6730d2a0f6b0f6241eabfffeb153ffffb9feffffffffaa9f");
  fp2_from_hex(&ISO_XDEN[2], "1", "0");
  fp2_from_hex(&ISO_YNUM[0], "1530477c7ab4113b59a4c18b076d11930f7da5d4a07f649bf54439d87d27e500fc8c25ebf8c92f6812cfc71c71c6d706",
               "1530477c7ab4113b59a4c18b076d11930f7da5d4a07f649bf54439d87d27e500fc8c25ebf8c92f6812cfc71c71c6d706");
  fp2_from_hex(&ISO_YNUM[1], "0", "5c759507e8e333ebb5b7a9a47d7ed8532c52d39fd3a042a88b58423c50ae15d5c2638e343d9c71c6238aaaaaaaa97be");
  fp2_from_hex(&ISO_YNUM[2], "11560bf17baa99bc32126fced787c88f984f87adf7ae0c7f9a208c6b4f20a4181472aaa9cb8d555526a9ffffffffc71c",
               "8ab05f8bdd54cde190937e76bc3e447cc27c3d6fbd7063fcd104635a790520c0a395554e5c6aaaa9354ffffffffe38f");
  fp2_from_hex(&ISO_YNUM[3], "124c9ad43b6cf79bfbf7043de3811ad0761b0f37a1e26286b0e977c69aa274524e79097a56dc4bd9e1b371c71c718b10", "0");
  fp2_from_hex(&ISO_YDEN[0], "1a0111ea397fe69a4b1ba7b6434bacd764774b84f38512bf6730d2a0f6b0f6241eabfffeb153ffffb9feffffffffa8fb",
               "1a0111ea397fe69a4b1ba7b6434bacd764774b84f38512bf6730d2a0f6b0f6241eabfffeb153ffffb9feffffffffa8fb");
  fp2_from_hex(&ISO_YDEN[1], "0", "1a0111ea397fe69a4b1ba7b6434bacd764774b84f38512bf6730d2a0f6b0f6241eabfffeb153ffffb9feffffffffa9d3");
  fp2_from_hex(&ISO_YDEN[2], "12", "1a0111ea397fe69a4b1ba7b6434bacd764774b84f38512bf6730d2a0f6b0f6241eabfffeb153ffffb9feffffffffaa99");
  fp2_from_hex(&ISO_YDEN[3], "1", "0");
  g_inited = 1;
}
void twin_init(void) { pthread_once(&g_once, do_init); }

/* ------------------------------------------------------------------------------------------ Fr */
static void scalar_from_be32(u64 k[4], const uint8_t* b) {
  for (int i = 0; i < 4; ++i) {
    u64 v = 0;
    for (int j = 0; j < 8; ++j) v = (v << 8) | b[(3 - i) * 8 + j];
    k[i] = v;
  }
}
static void fr_reduce(u64 k[4]) { /* k < 2^256 < 3r: subtract r while >= r */
  for (int it = 0; it < 3; ++it) {
    int ge = 1;
    for (int i = 3; i >= 0; --i) {
      if (k[i] > R_ORD[i]) { ge = 1; break; }
      if (k[i] < R_ORD[i]) { ge = 0; break; }
    }
    if (!ge) return;
    u64 br = 0;
    for (int i = 0; i < 4; ++i) {
      u128 d = (u128)k[i] - R_ORD[i] - br;
      k[i] = (u64)d;
      br = (u64)(d >> 64) & 1;
    }
  }
}
/* plain modular arithmetic mod r via u128 schoolbook + long reduction (slow, only O(t^2) per Recover) */
static void fr_mulmod(u64 r[4], const u64 a[4], const u64 b[4]) {
  u64 t[8] = {0};
  for (int i = 0; i < 4; ++i) {
    u64 c = 0;
    for (int j = 0; j < 4; ++j) {
      u128 s = (u128)a[i] * b[j] + t[i + j] + c;
      t[i + j] = (u64)s;
      c = (u64)(s >> 64);
    }
    t[i + 4] = c;
  }
  /* binary long reduction of 512-bit t mod r */
  u64 rem[5] = {0};
  for (int bit = 511; bit >= 0; --bit) {
    /* rem = rem*2 + bit */
    u64 carry = (t[bit / 64] >> (bit % 64)) & 1;
    for (int i = 0; i < 5; ++i) {
      u64 nc = rem[i] >> 63;
      rem[i] = (rem[i] << 1) | carry;
      carry = nc;
    }
    int ge = rem[4] != 0;
    if (!ge) {
      ge = 1;
      for (int i = 3; i >= 0; --i) {
        if (rem[i] > R_ORD[i]) { ge = 1; break; }
        if (rem[i] < R_ORD[i]) { ge = 0; break; }
      }
    }
    if (ge) {
      u64 br = 0;
      for (int i = 0; i < 4; ++i) {
        u128 d = (u128)rem[i] - R_ORD[i] - br;
        rem[i] = (u64)d;
        br = (u64)(d >> 64) & 1;
      }
      rem[4] -= br;
    }
  }
  memcpy(r, rem, 32);
}
static void fr_sub(u64 r[4], const u64 a[4], const u64 b[4]) {
  u64 br = 0, t[4];
  for (int i = 0; i < 4; ++i) {
    u128 d = (u128)a[i] - b[i] - br;
    t[i] = (u64)d;
    br = (u64)(d >> 64) & 1;
  }
  if (br) {
    u64 c = 0;
    for (int i = 0; i < 4; ++i) {
      u128 s = (u128)t[i] + R_ORD[i] + c;
      t[i] = (u64)s;
      c = (u64)(s >> 64);
    }
  }
  memcpy(r, t, 32);
}
static void fr_inv(u64 r[4], const u64 a[4]) {
  u64 e[4];
  memcpy(e, R_ORD, 32);
  e[0] -= 2;
  u64 acc[4] = {1, 0, 0, 0};
  for (int i = 3; i >= 0; --i)
    for (int b = 63; b >= 0; --b) {
      fr_mulmod(acc, acc, acc);
      if ((e[i] >> b) & 1) fr_mulmod(acc, acc, a);
    }
  memcpy(r, acc, 32);
}

/* ------------------------------------------------------------------------------------------ API */
void twin_hash_to_g2(const uint8_t* msg, size_t msg_len, const uint8_t* dst, size_t dst_len, uint8_t out96[96]) {
  twin_init();
  g2j h;
  hash_to_g2_point(&h, msg, msg_len, dst, dst_len);
  g2_compress(out96, &h);
}
void twin_sign(const uint8_t sk32[32], const uint8_t* msg, size_t msg_len, uint8_t out96[96]) {
  twin_init();
  u64 k[4];
  scalar_from_be32(k, sk32);
  fr_reduce(k);
  g2j h, s;
  size_t dl;
  const uint8_t* dst = cur_dst(&dl);
  hash_to_g2_point(&h, msg, msg_len, dst, dl);
  g2_mul(&s, &h, k, 4);
  g2_compress(out96, &s);
}
static int verify_point(const g1j* pk, const uint8_t* msg, size_t msg_len, const uint8_t sig96[96]) {
  g2j s, h;
  if (!g2_decompress(&s, sig96)) return 2;
  size_t dl;
  const uint8_t* dst = cur_dst(&dl);
  hash_to_g2_point(&h, msg, msg_len, dst, dl);
  /* e(pk, H) * e(-g1, sig) == 1 */
  fp px[2], py[2];
  fp2 qx[2], qy[2];
  int np = 0;
  int pk_inf = fp_is_zero(&pk->z), h_inf = fp2_is_zero(&h.z), s_inf = fp2_is_zero(&s.z);
  if (!pk_inf && !h_inf) {
    g1_to_affine(&px[np], &py[np], pk);
    g2_to_affine(&qx[np], &qy[np], &h);
    ++np;
  }
  if (!s_inf) {
    /* -g1 */
    static const char* gx = "17f1d3a73197d7942695638c4fa9ac0fc3688c4f9774b905a14e3a3f171bac586c55e83ff97a1aeffb3af00adb22c6bb";
    static const char* gy = "08b3f481e3aaa0f1a09e30ed741d8ae4fcf5e095d5d00af600db18cb2c04b3edd03cc744a2888ae40caa232946c5e7e1";
    fp_from_hex(&px[np], gx);
    fp_from_hex(&py[np], gy);
    fp_neg(&py[np], &py[np]);
    g2_to_affine(&qx[np], &qy[np], &s);
    ++np;
  }
  if (np == 0) return 0;
  fp12 f, r;
  miller_loop_multi(&f, np, px, py, qx, qy);
  final_exp(&r, &f);
  return fp12_is_one(&r) ? 0 : 1;
}
int twin_verify(const uint8_t pk48[48], const uint8_t* msg, size_t msg_len, const uint8_t sig96[96]) {
  twin_init();
  g1j pk;
  if (!g1_decompress(&pk, pk48)) return 4;
  return verify_point(&pk, msg, msg_len, sig96);
}
typedef struct {
  const g1j* pk;
  const uint8_t* msgs;
  size_t msg_len;
  const uint8_t* sigs;
  uint8_t* status;
  size_t lo, hi;
} vjob;
static void* verify_worker(void* arg) {
  vjob* j = (vjob*)arg;
  for (size_t i = j->lo; i < j->hi; ++i)
    j->status[i] = (uint8_t)verify_point(j->pk, j->msgs + i * j->msg_len, j->msg_len, j->sigs + 96 * i);
  return NULL;
}
void twin_verify_batch(const uint8_t pk48[48], size_t n, const uint8_t* msgs, size_t msg_len, const uint8_t* sigs96,
                       uint8_t* status, int threads) {
  twin_init();
  g1j pk;
  if (!g1_decompress(&pk, pk48)) {
    memset(status, 4, n);
    return;
  }
  if (threads < 1) threads = 1;
  pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * threads);
  vjob* jobs = (vjob*)malloc(sizeof(vjob) * threads);
  for (int t = 0; t < threads; ++t) {
    jobs[t] = (vjob){&pk, msgs, msg_len, sigs96, status, n * t / threads, n * (t + 1) / threads};
    pthread_create(&th[t], NULL, verify_worker, &jobs[t]);
  }
  for (int t = 0; t < threads; ++t) pthread_join(th[t], NULL);
  free(th);
  free(jobs);
}
void twin_beacon_message(const uint8_t* prev_sig, size_t prev_sig_len, uint64_t prev_round, uint64_t round,
                         uint8_t out32[32]) {
  uint8_t b[8];
  sha256_ctx c;
  sha256_init(&c);
  for (int i = 0; i < 8; ++i) b[i] = (uint8_t)(prev_round >> (56 - 8 * i));
  sha256_update(&c, b, 8);
  sha256_update(&c, prev_sig, prev_sig_len);
  for (int i = 0; i < 8; ++i) b[i] = (uint8_t)(round >> (56 - 8 * i));
  sha256_update(&c, b, 8);
  sha256_final(&c, out32);
}
void twin_gen_chain(const uint8_t sk32[32], const uint8_t* seed, size_t seed_len, uint64_t first_round, size_t n,
                    uint8_t* out_sigs96) {
  twin_init();
  const uint8_t* prev = seed;
  size_t prev_len = seed_len;
  for (size_t i = 0; i < n; ++i) {
    uint8_t msg[32];
    uint64_t r = first_round + i;
    twin_beacon_message(prev, prev_len, r - 1, r, msg);
    twin_sign(sk32, msg, 32, out_sigs96 + 96 * i);
    prev = out_sigs96 + 96 * i;
    prev_len = 96;
  }
}
static int pubpoly_eval_point(g1j* out, const uint8_t* commits48, uint32_t t, uint32_t index) {
  g1j acc;
  memset(&acc, 0, sizeof acc);
  u64 x[1] = {(u64)index + 1};
  for (int j = (int)t - 1; j >= 0; --j) {
    g1j c;
    if (!g1_decompress(&c, commits48 + 48 * j)) return 4;
    g1_mul(&acc, &acc, x, 1);
    g1_add(&acc, &acc, &c);
  }
  *out = acc;
  return 0;
}
int twin_pubpoly_eval(const uint8_t* commits48, uint32_t t, uint32_t index, uint8_t out48[48]) {
  twin_init();
  g1j p;
  int st = pubpoly_eval_point(&p, commits48, t, index);
  if (st) return st;
  g1_compress(out48, &p);
  return 0;
}
void twin_g1_mul_gen(const uint8_t sk32[32], uint8_t out48[48]) {
  twin_init();
  g1j g;
  fp_from_hex(&g.x, "17f1d3a73197d7942695638c4fa9ac0fc3688c4f9774b905a14e3a3f171bac586c55e83ff97a1aeffb3af00adb22c6bb");
  fp_from_hex(&g.y, "08b3f481e3aaa0f1a09e30ed741d8ae4fcf5e095d5d00af600db18cb2c04b3edd03cc744a2888ae40caa232946c5e7e1");
  g.z = FP_ONE;
  u64 k[4];
  scalar_from_be32(k, sk32);
  fr_reduce(k);
  g1j r;
  g1_mul(&r, &g, k, 4);
  g1_compress(out48, &r);
}
int twin_verify_partial(const uint8_t* commits48, uint32_t t, const uint8_t* msg, size_t msg_len,
                        const uint8_t* partial, size_t partial_len) {
  twin_init();
  if (partial_len < 2) return 3;
  if (partial_len != 98) return 2;
  uint32_t idx = (uint32_t)partial[0] << 8 | partial[1];
  g1j x;
  if (pubpoly_eval_point(&x, commits48, t, idx)) return 4;
  return verify_point(&x, msg, msg_len, partial + 2);
}
int twin_recover(const uint8_t* commits48, uint32_t t, uint32_t n, const uint8_t* msg, size_t msg_len,
                 const uint8_t* partials98, uint32_t k, uint8_t out96[96], uint8_t* share_status) {
  twin_init();
  (void)n;
  memset(share_status, 255, k);
  uint32_t* idx = (uint32_t*)malloc(sizeof(uint32_t) * (t + 1));
  uint32_t* pos = (uint32_t*)malloc(sizeof(uint32_t) * (t + 1));
  uint32_t got = 0;
  for (uint32_t s = 0; s < k && got < t; ++s) {
    int st = twin_verify_partial(commits48, t, msg, msg_len, partials98 + 98 * (size_t)s, 98);
    share_status[s] = (uint8_t)st;
    if (st) continue;
    idx[got] = (uint32_t)partials98[98 * (size_t)s] << 8 | partials98[98 * (size_t)s + 1];
    pos[got] = s;
    ++got;
  }
  /* xyCommit: sort by index, collapse duplicates */
  for (uint32_t a = 1; a < got; ++a)
    for (uint32_t b = a; b > 0 && idx[b - 1] > idx[b]; --b) {
      uint32_t ti = idx[b]; idx[b] = idx[b - 1]; idx[b - 1] = ti;
      uint32_t tp = pos[b]; pos[b] = pos[b - 1]; pos[b - 1] = tp;
    }
  uint32_t m = 0;
  for (uint32_t a = 0; a < got; ++a)
    if (m == 0 || idx[m - 1] != idx[a]) { idx[m] = idx[a]; pos[m] = pos[a]; ++m; }
  int rs = 0;
  if (m < t) {
    rs = 5;
    memset(out96, 0, 96);
  } else {
    g2j acc;
    memset(&acc, 0, sizeof acc);
    for (uint32_t a = 0; a < m; ++a) {
      u64 num[4] = {1, 0, 0, 0}, den[4] = {1, 0, 0, 0};
      u64 xi[4] = {(u64)idx[a] + 1, 0, 0, 0};
      for (uint32_t b = 0; b < m; ++b) {
        if (a == b) continue;
        u64 xj[4] = {(u64)idx[b] + 1, 0, 0, 0}, d[4];
        fr_mulmod(num, num, xj);
        fr_sub(d, xj, xi);
        fr_mulmod(den, den, d);
      }
      fr_inv(den, den);
      fr_mulmod(num, num, den);
      g2j s, term;
      g2_decompress(&s, partials98 + 98 * (size_t)pos[a] + 2);
      g2_mul(&term, &s, num, 4);
      g2_add(&acc, &acc, &term);
    }
    g2_compress(out96, &acc);
  }
  free(idx);
  free(pos);
  return rs;
}
typedef struct {
  const uint8_t* commits;
  uint32_t t, n, k;
  const uint8_t* msgs;
  const uint8_t* partials;
  uint8_t *out, *rs, *ss;
  size_t lo, hi;
} rjob;
static void* recover_worker(void* arg) {
  rjob* j = (rjob*)arg;
  for (size_t r = j->lo; r < j->hi; ++r)
    j->rs[r] = (uint8_t)twin_recover(j->commits, j->t, j->n, j->msgs + 32 * r, 32, j->partials + 98 * (size_t)j->k * r,
                                     j->k, j->out + 96 * r, j->ss + (size_t)j->k * r);
  return NULL;
}
void twin_recover_batch(const uint8_t* commits48, uint32_t t, uint32_t n, size_t rounds, const uint8_t* msgs32,
                        const uint8_t* partials98, uint32_t k, uint8_t* out96, uint8_t* round_status,
                        uint8_t* share_status, int threads) {
  twin_init();
  if (threads < 1) threads = 1;
  pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * threads);
  rjob* jobs = (rjob*)malloc(sizeof(rjob) * threads);
  for (int q = 0; q < threads; ++q) {
    jobs[q] = (rjob){commits48, t, n, k, msgs32, partials98, out96, round_status, share_status,
                     rounds * q / threads, rounds * (q + 1) / threads};
    pthread_create(&th[q], NULL, recover_worker, &jobs[q]);
  }
  for (int q = 0; q < threads; ++q) pthread_join(th[q], NULL);
  free(th);
  free(jobs);
}
int twin_pairing_cubed(const uint8_t g1_48[48], const uint8_t g2_96[96], uint8_t out576[576]) {
  twin_init();
  g1j p;
  g2j q;
  if (!g1_decompress(&p, g1_48)) return 4;
  if (!g2_decompress(&q, g2_96)) return 2;
  fp px, py;
  fp2 qx, qy;
  fp12 f, r;
  if (fp_is_zero(&p.z) || fp2_is_zero(&q.z)) {
    r = FP12_ONE;
  } else {
    g1_to_affine(&px, &py, &p);
    g2_to_affine(&qx, &qy, &q);
    miller_loop_multi(&f, 1, &px, &py, &qx, &qy);
    final_exp(&r, &f);
  }
  const fp2* slots[6] = {&r.c0.c0, &r.c0.c1, &r.c0.c2, &r.c1.c0, &r.c1.c1, &r.c1.c2};
  for (int i = 0; i < 6; ++i) {
    fp_to_be(out576 + 96 * i, &slots[i]->c0);
    fp_to_be(out576 + 96 * i + 48, &slots[i]->c1);
  }
  return 0;
}
int twin_set_dst(const uint8_t* dst, size_t dst_len) {
  if (dst_len > 255) return -1;
  if (dst == NULL || dst_len == 0) {
    g_dst_len = 0;
    return 0;
  }
  memcpy(g_dst, dst, dst_len);
  g_dst_len = dst_len;
  return 0;
}
typedef struct {
  const uint8_t *commits, *shares, *msgs;
  uint32_t t, n;
  uint8_t* out;
  size_t lo, hi, ok;
} c1job;
static void* c1_worker(void* arg) {
  c1job* j = (c1job*)arg;
  uint8_t* parts = (uint8_t*)malloc(98 * (size_t)j->n);
  uint8_t* ss = (uint8_t*)malloc(j->n);
  for (size_t r = j->lo; r < j->hi; ++r) {
    const uint8_t* msg = j->msgs + 32 * r;
    for (uint32_t i = 0; i < j->n; ++i) { /* tbls.Sign of every node (beacon/beacon.go:433) */
      parts[98 * i] = (uint8_t)(i >> 8);
      parts[98 * i + 1] = (uint8_t)i;
      twin_sign(j->shares + 32 * i, msg, 32, parts + 98 * i + 2);
    }
    /* Recover (beacon/beacon.go:488) then VerifyRecovered against pub.Commit() (:494) */
    if (twin_recover(j->commits, j->t, j->n, msg, 32, parts, j->n, j->out + 96 * r, ss) == 0 &&
        twin_verify(j->commits, msg, 32, j->out + 96 * r) == 0)
      ++j->ok;
  }
  free(parts);
  free(ss);
  return NULL;
}
size_t twin_c1_batch(const uint8_t* commits48, uint32_t t, uint32_t n, const uint8_t* shares32, size_t rounds,
                     const uint8_t* msgs32, uint8_t* out96, int threads) {
  twin_init();
  if (threads < 1) threads = 1;
  pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * threads);
  c1job* jobs = (c1job*)malloc(sizeof(c1job) * threads);
  for (int q = 0; q < threads; ++q) {
    jobs[q] = (c1job){commits48, shares32, msgs32, t, n, out96, rounds * q / threads, rounds * (q + 1) / threads, 0};
    pthread_create(&th[q], NULL, c1_worker, &jobs[q]);
  }
  size_t ok = 0;
  for (int q = 0; q < threads; ++q) {
    pthread_join(th[q], NULL);
    ok += jobs[q].ok;
  }
  free(th);
  free(jobs);
  return ok;
}
void twin_opcount_reset(void) { g_count = 0; }
uint64_t twin_opcount(void) { return g_count; }
void twin_opcount_enable(int on) { g_count_on = on; (void)g_count_total; (void)g_count_mu; (void)g_inited; }
