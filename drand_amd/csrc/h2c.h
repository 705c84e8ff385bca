// SHA-256, drand's beacon message (A1), randomness (A2) and RFC 9380 hash_to_curve for G2 (A9):
// BLS12381G2_XMD:SHA-256_SSWU_RO_ with the DST passed in (drand: BLS_SIG_BLS12381G2_XMD:SHA-256_SSWU_RO_NUL_,
// SURVEY.md §8(c); the variant is one switch: the DST bytes).
//   beacon.Message            beacon/chain.go:86-94 (roundToBytes beacon/store.go:248-252)
//   RandomnessFromSignature   beacon/chain.go:52-55
#pragma once
#include "curve.h"

namespace dg {

struct Sha256 {
  uint32_t h[8];
  uint32_t w[16];  // current block as big-endian words
  uint32_t len;    // bytes in current block
  uint32_t total;  // total bytes
};

DGI uint32_t rotr32(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }

DGH void sha256_compress(uint32_t h[8], const uint32_t* win) {
  const uint32_t K[64] = {
      0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5, 0xd807aa98,
      0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174, 0xe49b69c1, 0xefbe4786,
      0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da, 0x983e5152, 0xa831c66d, 0xb00327c8,
      0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967, 0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13,
      0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85, 0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819,
      0xd6990624, 0xf40e3585, 0x106aa070, 0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a,
      0x5b9cca4f, 0x682e6ff3, 0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7,
      0xc67178f2};
  uint32_t w[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) w[i] = win[i];
  uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], hh = h[7];
#pragma unroll
  for (int i = 0; i < 64; ++i) {
    uint32_t wi;
    if (i < 16) {
      wi = w[i];
    } else {
      uint32_t w15 = w[(i + 1) & 15], w2 = w[(i + 14) & 15];
      uint32_t s0 = rotr32(w15, 7) ^ rotr32(w15, 18) ^ (w15 >> 3);
      uint32_t s1 = rotr32(w2, 17) ^ rotr32(w2, 19) ^ (w2 >> 10);
      wi = w[i & 15] + s0 + w[(i + 9) & 15] + s1;
      w[i & 15] = wi;
    }
    uint32_t t1 = hh + (rotr32(e, 6) ^ rotr32(e, 11) ^ rotr32(e, 25)) + ((e & f) ^ (~e & g)) + K[i] + wi;
    uint32_t t2 = (rotr32(a, 2) ^ rotr32(a, 13) ^ rotr32(a, 22)) + ((a & b) ^ (a & c) ^ (b & c));
    hh = g;
    g = f;
    f = e;
    e = d + t1;
    d = c;
    c = b;
    b = a;
    a = t1 + t2;
  }
  h[0] += a;
  h[1] += b;
  h[2] += c;
  h[3] += d;
  h[4] += e;
  h[5] += f;
  h[6] += g;
  h[7] += hh;
}

DGI void sha256_init(Sha256& s) {
  const uint32_t iv[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a, 0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
  for (int i = 0; i < 8; ++i) s.h[i] = iv[i];
  for (int i = 0; i < 16; ++i) s.w[i] = 0;
  s.len = 0;
  s.total = 0;
}
DGI void sha256_byte(Sha256& s, uint8_t v) {
  uint32_t wi = s.len >> 2, sh = 24 - 8 * (s.len & 3);
  s.w[wi] |= (uint32_t)v << sh;
  s.len++;
  s.total++;
  if (s.len == 64) {
    sha256_compress(s.h, s.w);
    for (int i = 0; i < 16; ++i) s.w[i] = 0;
    s.len = 0;
  }
}
DGI void sha256_update(Sha256& s, const uint8_t* d, uint32_t n) {
  for (uint32_t i = 0; i < n; ++i) sha256_byte(s, d[i]);
}
DGI void sha256_update_zeros(Sha256& s, uint32_t n) {
  for (uint32_t i = 0; i < n; ++i) sha256_byte(s, 0);
}
DGI void sha256_final(Sha256& s, uint8_t out[32]) {
  uint64_t bits = (uint64_t)s.total * 8;
  sha256_byte(s, 0x80);
  while (s.len != 56) sha256_byte(s, 0);
  for (int i = 7; i >= 0; --i) sha256_byte(s, (uint8_t)(bits >> (8 * i)));
  for (int i = 0; i < 8; ++i) {
    out[4 * i] = (uint8_t)(s.h[i] >> 24);
    out[4 * i + 1] = (uint8_t)(s.h[i] >> 16);
    out[4 * i + 2] = (uint8_t)(s.h[i] >> 8);
    out[4 * i + 3] = (uint8_t)s.h[i];
  }
}

// beacon.Message: SHA256(BE64(prevRound) || prevSig || BE64(round))
DGI void beacon_message(uint8_t out[32], const uint8_t* prev_sig, uint32_t prev_sig_len, uint64_t prev_round,
                        uint64_t round) {
  Sha256 s;
  sha256_init(s);
  for (int i = 7; i >= 0; --i) sha256_byte(s, (uint8_t)(prev_round >> (8 * i)));
  sha256_update(s, prev_sig, prev_sig_len);
  for (int i = 7; i >= 0; --i) sha256_byte(s, (uint8_t)(round >> (8 * i)));
  sha256_final(s, out);
}

// RFC 9380 §5.3.1 expand_message_xmd(msg, DST, 256) -> hash_to_field (count 2, m 2, L 64).
DGH void hash_to_field_fp2x2(Fp2 u[2], const uint8_t* msg, uint32_t msg_len, const uint8_t* dst, uint32_t dst_len) {
  uint8_t b0[32], bi[32];
  Sha256 s;
  sha256_init(s);
  sha256_update_zeros(s, 64);
  sha256_update(s, msg, msg_len);
  sha256_byte(s, 1);  // l_i_b_str = I2OSP(256, 2)
  sha256_byte(s, 0);
  sha256_byte(s, 0);  // I2OSP(0, 1)
  sha256_update(s, dst, dst_len);
  sha256_byte(s, (uint8_t)dst_len);
  sha256_final(s, b0);
  uint8_t chunk[64];
  for (int i = 1; i <= 8; ++i) {
    sha256_init(s);
    if (i == 1) {
      sha256_update(s, b0, 32);
    } else {
      for (int k = 0; k < 32; ++k) sha256_byte(s, b0[k] ^ bi[k]);
    }
    sha256_byte(s, (uint8_t)i);
    sha256_update(s, dst, dst_len);
    sha256_byte(s, (uint8_t)dst_len);
    sha256_final(s, bi);
    // uniform bytes [32(i-1), 32 i): element e = (i-1)/2, half = (i-1)%2
    int half = (i - 1) & 1;
    for (int k = 0; k < 32; ++k) chunk[32 * half + k] = bi[k];
    if (half == 1) {
      int e = (i - 1) >> 1;  // 0: u0.c0, 1: u0.c1, 2: u1.c0, 3: u1.c1
      Fp v = fp_from_be64(chunk);
      if (e == 0) u[0].c0 = v;
      else if (e == 1) u[0].c1 = v;
      else if (e == 2) u[1].c0 = v;
      else u[1].c1 = v;
    }
  }
}

// ---- expand_message_xmd for 32-byte messages, word-wise (drand hashes 32 B SHA-256 outputs).  The host
// builds the message-independent words of every SHA-256 block (xmd_tail_build: the state after b_0's
// all-zero first block, then the padded DST tails); the device streams 32-bit words with static indices,
// no byte arrays.  Same bytes as hash_to_field_fp2x2 (RFC 9380 §5.3.1, L = 64, count 2, m 2).
constexpr int XMD_MAXB = 5;  // SHA-256 blocks per hash for DST lengths up to 255
struct XmdTail {
  uint32_t nb0, nbi;                // blocks of b_0 after its zero block; blocks of each b_i
  uint32_t h_zero[8];               // state after the 64-byte zero block of b_0
  uint32_t w0[XMD_MAXB * 16];       // b_0's blocks: words 0..7 of the first one are the message
  uint32_t wi[8][XMD_MAXB * 16];    // b_i's blocks: words 0..7 of the first one are b_0 ^ b_{i-1}
};

static inline void xmd_tail_build(XmdTail& T, const uint8_t* dst, uint32_t dst_len) {
  const uint32_t iv[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a, 0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
  uint8_t buf[XMD_MAXB * 64 + 64];
  auto words = [](const uint8_t* b, uint32_t* w, int n) {
    for (int t = 0; t < n; ++t)
      w[t] = (uint32_t)b[4 * t] << 24 | (uint32_t)b[4 * t + 1] << 16 | (uint32_t)b[4 * t + 2] << 8 | b[4 * t + 3];
  };
  // padded message of `len` bytes already in buf -> number of blocks
  auto pad = [&](uint32_t len) {
    uint32_t nb = (len + 9 + 63) / 64;
    for (uint32_t k = len; k < nb * 64; ++k) buf[k] = 0;
    buf[len] = 0x80;
    uint64_t bits = (uint64_t)len * 8;
    for (int k = 0; k < 8; ++k) buf[nb * 64 - 1 - k] = (uint8_t)(bits >> (8 * k));
    return nb;
  };
  for (int k = 0; k < 8; ++k) T.h_zero[k] = iv[k];
  uint32_t zw[16] = {0};
  sha256_compress(T.h_zero, zw);
  // b_0 = H(Z_pad || msg || I2OSP(256, 2) || I2OSP(0, 1) || DST || I2OSP(len(DST), 1)), after the zero block
  uint32_t len = 0;
  for (int k = 0; k < 32; ++k) buf[len++] = 0;  // the message's place
  buf[len++] = 1;
  buf[len++] = 0;
  buf[len++] = 0;
  for (uint32_t k = 0; k < dst_len; ++k) buf[len++] = dst[k];
  buf[len++] = (uint8_t)dst_len;
  // the length field counts the zero block too: pad as if 64 bytes preceded
  uint32_t nb = (len + 64 + 9 + 63) / 64 - 1;
  for (uint32_t k = len; k < nb * 64; ++k) buf[k] = 0;
  buf[len] = 0x80;
  uint64_t bits = (uint64_t)(len + 64) * 8;
  for (int k = 0; k < 8; ++k) buf[nb * 64 - 1 - k] = (uint8_t)(bits >> (8 * k));
  T.nb0 = nb;
  for (uint32_t k = 0; k < XMD_MAXB * 16; ++k) T.w0[k] = 0;
  words(buf, T.w0, (int)nb * 16);
  // b_i = H((b_0 xor b_{i-1}) || I2OSP(i, 1) || DST || I2OSP(len(DST), 1))
  for (int i = 1; i <= 8; ++i) {
    len = 0;
    for (int k = 0; k < 32; ++k) buf[len++] = 0;
    buf[len++] = (uint8_t)i;
    for (uint32_t k = 0; k < dst_len; ++k) buf[len++] = dst[k];
    buf[len++] = (uint8_t)dst_len;
    nb = pad(len);
    T.nbi = nb;
    for (uint32_t k = 0; k < XMD_MAXB * 16; ++k) T.wi[i - 1][k] = 0;
    words(buf, T.wi[i - 1], (int)nb * 16);
  }
}

// nb SHA-256 blocks into h: words 0..7 of the first block from `head`, the rest from the host-built tail
DGI void xmd_blocks(uint32_t (&h)[8], const uint32_t (&head)[8], const uint32_t* tail, uint32_t nb) {
  uint32_t w[16];
  for (uint32_t blk = 0; blk < nb; ++blk) {
#pragma unroll
    for (int t = 0; t < 16; ++t) w[t] = (blk == 0 && t < 8) ? head[t] : tail[blk * 16 + t];
    sha256_compress(h, w);
  }
}

// 64 uniform bytes (big-endian words b_{2e+1} || b_{2e+2}) -> Fp: hi 2^256 + lo mod p, in Montgomery form
DGI Fp fp_from_words64(const uint32_t (&hi)[8], const uint32_t (&lo)[8]) {
  Fp a = fp_zero(), b = fp_zero();
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    a.l[k] = hi[7 - k];
    b.l[k] = lo[7 - k];
  }
  return fp_add(fp_mul(a, fp_const(FP_R2_2POW256)), fp_mul(b, fp_const(FP_R2)));
}

DGH void hash_to_field_xmd32(Fp2 u[2], const uint8_t* msg, const XmdTail* T) {
  const uint32_t iv[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a, 0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
  uint32_t m[8], h[8], b0[8], bp[8], v[8];
#pragma unroll
  for (int t = 0; t < 8; ++t) {
    m[t] = (uint32_t)msg[4 * t] << 24 | (uint32_t)msg[4 * t + 1] << 16 | (uint32_t)msg[4 * t + 2] << 8 | msg[4 * t + 3];
    h[t] = T->h_zero[t];
  }
  xmd_blocks(h, m, T->w0, T->nb0);
#pragma unroll
  for (int t = 0; t < 8; ++t) {
    b0[t] = h[t];
    bp[t] = 0;
  }
  Fp e0 = fp_zero(), e1 = fp_zero(), e2 = fp_zero(), e3 = fp_zero();
#pragma unroll 1
  for (uint32_t i = 1; i <= 8; ++i) {
#pragma unroll
    for (int t = 0; t < 8; ++t) {
      v[t] = b0[t] ^ bp[t];  // b_0 xor b_{i-1} (b_0 alone for i = 1: bp = 0)
      h[t] = iv[t];
    }
    xmd_blocks(h, v, T->wi[i - 1], T->nbi);
    if ((i & 1) == 0) {
      Fp e = fp_from_words64(bp, h);
      e0 = fp_sel(i == 2, e0, e);
      e1 = fp_sel(i == 4, e1, e);
      e2 = fp_sel(i == 6, e2, e);
      e3 = fp_sel(i == 8, e3, e);
    }
#pragma unroll
    for (int t = 0; t < 8; ++t) bp[t] = h[t];
  }
  u[0] = Fp2{e0, e1};
  u[1] = Fp2{e2, e3};
}

// RFC 9380 §6.6.2 simplified SWU onto E2': y^2 = x^3 + A'x + B', A' = 240u, B' = 1012(1+u), Z = -(2+u).
// One Fp inversion, one Fp sqrt of the norm and one (p-3)/4 exponentiation; the gx2 branch reuses the
// first norm root through sqrt(norm(gx2)) = norm(u)^3 * 5 * sqrt(-5) * sqrt(-norm(gx1)).
DGH void sswu_g2(Fp2& ox, Fp2& oy, const Fp2& u, const Fp& den_inv_norm_hint, bool use_hint) {
  (void)den_inv_norm_hint;
  (void)use_hint;
  Fp2 A = fp2_const(SSWU_A), B = fp2_const(SSWU_B), Z = fp2_const(SSWU_Z);
  Fp2 u2 = fp2_sqr(u);
  Fp2 zu2 = fp2_mul(Z, u2);
  Fp2 den = fp2_add(fp2_sqr(zu2), zu2);
  Fp2 x1;
  if (fp2_is_zero(den)) {
    x1 = fp2_const(SSWU_B_OVER_ZA);
  } else {
    x1 = fp2_mul(fp2_const(SSWU_MINUS_B_OVER_A), fp2_add(fp2_one(), fp2_inv(den)));
  }
  Fp2 gx1 = fp2_add(fp2_mul(fp2_add(fp2_sqr(x1), A), x1), B);
  Fp n1 = fp2_norm(gx1);
  Fp t = fp_pow_pm3d4(n1);
  Fp s1 = fp_mul(t, n1);  // n1^((p+1)/4)
  bool sq1 = fp_eq(fp_sqr(s1), n1);
  Fp2 x, g;
  Fp s;
  if (sq1) {
    x = x1;
    g = gx1;
    s = s1;
  } else {
    x = fp2_mul(zu2, x1);
    g = fp2_add(fp2_mul(fp2_add(fp2_sqr(x), A), x), B);
    // s1^2 = -n1 ; norm(gx2) = 5^3 norm(u)^6 n1 ; sqrt = norm(u)^3 * 5 * sqrt(-5) * s1
    Fp nu = fp2_norm(u);
    Fp nu3 = fp_mul(fp_sqr(nu), nu);
    s = fp_mul(fp_mul(nu3, fp_small(5)), fp_mul(fp_const(FP_SQRT_MINUS5), s1));
  }
  Fp2 y;
  bool ok = fp2_sqrt_with_norm_root(y, g, s);
  if (!ok) {
    // the shortcut root may carry the other sign: retry with -s
    fp2_sqrt_with_norm_root(y, g, fp_neg(s));
  }
  if (fp2_sgn0(u) != fp2_sgn0(y)) y = fp2_neg(y);
  ox = x;
  oy = y;
}

DGI Fp2 poly_eval_const(const uint32_t (*c)[2][12], int n, const Fp2& x) {
  Fp2 acc = fp2_const(c[n - 1]);
  for (int i = n - 2; i >= 0; --i) acc = fp2_add(fp2_mul(acc, x), fp2_const(c[i]));
  return acc;
}

// 3-isogeny E2' -> E2 (RFC 9380 Appendix E.3), output in Jacobian coordinates without inversion
DGH G2J iso_map_g2(const Fp2& x, const Fp2& y) {
  Fp2 xn = poly_eval_const(ISO_XNUM, 4, x);
  Fp2 xd = poly_eval_const(ISO_XDEN, 3, x);
  Fp2 yn = poly_eval_const(ISO_YNUM, 4, x);
  Fp2 yd = poly_eval_const(ISO_YDEN, 4, x);
  if (fp2_is_zero(xd) || fp2_is_zero(yd)) return jac_infinity<Fp2>();
  Fp2 z = fp2_mul(xd, yd);
  Fp2 yd2 = fp2_sqr(yd);
  Fp2 X = fp2_mul(xn, fp2_mul(yd2, xd));
  Fp2 Y = fp2_mul(fp2_mul(fp2_mul(fp2_sqr(z), xd), yn), y);
  return G2J{X, Y, z};
}

// hash_to_curve without the final clear_cofactor (the RLC batch applies h_eff once to the sum)
DGI G2J hash_to_g2_uncleared(const uint8_t* msg, uint32_t msg_len, const uint8_t* dst, uint32_t dst_len) {
  Fp2 u[2];
  hash_to_field_fp2x2(u, msg, msg_len, dst, dst_len);
  G2J q[2];
  for (int i = 0; i < 2; ++i) {
    Fp2 x, y;
    sswu_g2(x, y, u[i], fp_zero(), false);
    q[i] = iso_map_g2(x, y);
  }
  return jac_add(q[0], q[1]);
}
DGI G2J hash_to_g2(const uint8_t* msg, uint32_t msg_len, const uint8_t* dst, uint32_t dst_len) {
  return g2_clear_cofactor(hash_to_g2_uncleared(msg, msg_len, dst, dst_len));
}

}  // namespace dg
