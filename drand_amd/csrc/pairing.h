// Optimal-ate pairing on BLS12-381 (A11): Miller loop over |z| = 0xd201000000010000 with homogeneous
// projective G2 steps and sparse M-twist lines (slots 0, 1, 4 of Fp12 = Fp6[w]/(w^2 - v)), and the
// final exponentiation f^((p^6-1)(p^2+1)) followed by the hard part 3*Phi12(p)/r =
// (z-1)^2 (z+p)(z^2+p^2-1) + 3 (Hayashida-Hayasaka-Teruya).  The result is e(P,Q)^3, which is 1
// exactly when e(P,Q) is (3 does not divide r), the only use the verify path makes of it.
#pragma once
#include "curve.h"

namespace dg {

struct G2Proj {
  Fp2 x, y, z;
};

// DG_ML_INLINE=2 also inlines the line evaluations into the Miller loop (A/B)
#if defined(DG_ML_INLINE) && DG_ML_INLINE >= 2
DGI
#else
DG12
#endif
void line_dbl(G2Proj& T, Fp2& c0, Fp2& c1, Fp2& c4, const Fp& px, const Fp& py) {
  Fp2 a = fp2_mul_fp(fp2_mul(T.x, T.y), fp_const(FP_TWO_INV));
  Fp2 b = fp2_sqr(T.y);
  Fp2 c = fp2_sqr(T.z);
  Fp2 e = fp2_mul(fp2_const(FP2_B3_G2), c);
  Fp2 f = fp2_add(fp2_dbl(e), e);
  Fp2 g = fp2_mul_fp(fp2_add(b, f), fp_const(FP_TWO_INV));
  Fp2 h = fp2_sub(fp2_sub(fp2_sqr(fp2_add(T.y, T.z)), b), c);
  Fp2 j = fp2_sqr(T.x);
  c0 = fp2_sub(e, b);
  c1 = fp2_mul_fp(fp2_add(fp2_dbl(j), j), px);
  c4 = fp2_mul_fp(fp2_neg(h), py);
  Fp2 e2 = fp2_sqr(e);
  T.x = fp2_mul(a, fp2_sub(b, f));
  T.y = fp2_sub(fp2_sqr(g), fp2_add(fp2_dbl(e2), e2));
  T.z = fp2_mul(b, h);
}

#if defined(DG_ML_INLINE) && DG_ML_INLINE >= 2
DGI
#else
DG12
#endif
void line_add(G2Proj& T, const Fp2& qx, const Fp2& qy, Fp2& c0, Fp2& c1, Fp2& c4, const Fp& px, const Fp& py) {
  Fp2 theta = fp2_sub(T.y, fp2_mul(qy, T.z));
  Fp2 lambda = fp2_sub(T.x, fp2_mul(qx, T.z));
  Fp2 c = fp2_sqr(theta);
  Fp2 d = fp2_sqr(lambda);
  Fp2 e = fp2_mul(lambda, d);
  Fp2 f = fp2_mul(T.z, c);
  Fp2 g = fp2_mul(T.x, d);
  Fp2 h = fp2_sub(fp2_add(e, f), fp2_dbl(g));
  Fp2 ny = fp2_sub(fp2_mul(theta, fp2_sub(g, h)), fp2_mul(e, T.y));
  T.x = fp2_mul(lambda, h);
  T.y = ny;
  T.z = fp2_mul(T.z, e);
  c0 = fp2_sub(fp2_mul(theta, qx), fp2_mul(lambda, qy));
  c1 = fp2_mul_fp(fp2_neg(theta), px);
  c4 = fp2_mul_fp(lambda, py);
}

// prod_k f_{z,Q_k}(P_k) for up to NP pairs (affine inputs, none at infinity; callers drop such pairs)
template <int NP>
DGI Fp12 miller_loop(const G1A* P, const G2A* Q, int np) {
  G2Proj T[NP];
  for (int k = 0; k < NP; ++k)
    if (k < np) T[k] = G2Proj{Q[k].x, Q[k].y, fp2_one()};
  Fp12 f = fp12_one();
  for (int b = 62; b >= 0; --b) {
    f = fp12_sqr(f);
    for (int k = 0; k < NP; ++k) {
      if (k >= np) break;
      Fp2 c0, c1, c4;
      line_dbl(T[k], c0, c1, c4, P[k].x, P[k].y);
      f = fp12_mul_014(f, c0, c1, c4);
    }
    if ((Z_ABS >> b) & 1) {
      for (int k = 0; k < NP; ++k) {
        if (k >= np) break;
        Fp2 c0, c1, c4;
        line_add(T[k], Q[k].x, Q[k].y, c0, c1, c4, P[k].x, P[k].y);
        f = fp12_mul_014(f, c0, c1, c4);
      }
    }
  }
  return fp12_conj(f);  // z < 0
}

// Compressed cyclotomic squaring (Karabina, "Squaring in cyclotomic subgroups", Math. Comp. 2013): an element of
// the cyclotomic subgroup is determined by four of its six Fp2 coefficients, and squaring maps those four among
// themselves.  Naming as in fp12_cyc_sqr: g0 = c0.c0, g1 = c1.c1, g2 = c1.c0, g3 = c0.c2, g4 = c0.c1, g5 = c1.c2.
//   h2 = 2 g2 + 3 xi (2 g4 g5)          h3 = 3 (g4^2 + xi g5^2) - 2 g3
//   h4 = 3 (g2^2 + xi g3^2) - 2 g4      h5 = 2 g5 + 3 (2 g2 g3)
// six Fp2 squarings (2 g_i g_j = (g_i + g_j)^2 - g_i^2 - g_j^2) instead of Granger-Scott's nine.  Decompression
// (g2 != 0): g1 = (xi g5^2 + 3 g4^2 - 2 g3) / (4 g2), g0 = xi (2 g1^2 + g2 g5 - 3 g3 g4) + 1.
#ifndef DG_CYC_KARABINA
#define DG_CYC_KARABINA 1
#endif
struct CycC {
  Fp2 g2, g3, g4, g5;
};
DGI CycC cyc_sqr_c(const CycC& g) {
  const Fp2 s2 = DG_FP4_SQR2(g.g2), s3 = DG_FP4_SQR2(g.g3), s4 = DG_FP4_SQR2(g.g4), s5 = DG_FP4_SQR2(g.g5);
  const Fp2 b23 = fp2_sub(fp2_sub(DG_FP4_SQR2(fp2_add(g.g2, g.g3)), s2), s3);  // 2 g2 g3
  const Fp2 b45 = fp2_sub(fp2_sub(DG_FP4_SQR2(fp2_add(g.g4, g.g5)), s4), s5);  // 2 g4 g5
  const Fp2 t45 = fp2_mul_xi(b45);
  const Fp2 a45 = fp2_add(s4, fp2_mul_xi(s5));
  const Fp2 a23 = fp2_add(s2, fp2_mul_xi(s3));
  CycC h;
  h.g2 = fp2_add(fp2_dbl(g.g2), fp2_add(fp2_dbl(t45), t45));
  h.g3 = fp2_sub(fp2_add(fp2_dbl(a45), a45), fp2_dbl(g.g3));
  h.g4 = fp2_sub(fp2_add(fp2_dbl(a23), a23), fp2_dbl(g.g4));
  h.g5 = fp2_add(fp2_dbl(g.g5), fp2_add(fp2_dbl(b23), b23));
  return h;
}
// the full element from its compressed form, given inv = 1 / (4 g2)
DGI Fp12 cyc_decompress(const CycC& g, const Fp2& inv) {
  const Fp2 g44 = fp2_sqr(g.g4);
  const Fp2 num = fp2_sub(fp2_add(fp2_mul_xi(fp2_sqr(g.g5)), fp2_add(fp2_dbl(g44), g44)), fp2_dbl(g.g3));
  const Fp2 g1 = fp2_mul(num, inv);
  const Fp2 g34 = fp2_mul(g.g3, g.g4);
  const Fp2 t = fp2_sub(fp2_add(fp2_dbl(fp2_sqr(g1)), fp2_mul(g.g2, g.g5)), fp2_add(fp2_dbl(g34), g34));
  const Fp2 g0 = fp2_add(fp2_mul_xi(t), fp2_one());
  return Fp12{Fp6{g0, g.g4, g.g3}, Fp6{g.g2, g1, g.g5}};
}

// a^z for a in the cyclotomic subgroup (z < 0: conjugate of a^|z|), cyclotomic squarings
DG12 Fp12 cyc_exp_z(const Fp12& a) {
#if DG_CYC_KARABINA
  // |z| = 2^63 + 2^62 + 2^60 + 2^57 + 2^48 + 2^16: the six powers a^(2^k) by 63 compressed squarings, their
  // denominators inverted together (Montgomery's trick, one Fp2 inversion), then five products.  A zero
  // denominator (g2 = 0 at some power, e.g. a = 1) takes the uncompressed chain below.
  {
    constexpr int NB = 6;
    CycC s[NB];
    Fp2 pre[NB];
    CycC c{a.c1.c0, a.c0.c2, a.c0.c1, a.c1.c2};
    int n = 0;
    for (int k = 1; k <= 63; ++k) {
      c = cyc_sqr_c(c);
      if ((Z_ABS >> k) & 1) s[n++] = c;
    }
    bool zero = false;
    Fp2 run = fp2_one();
#pragma unroll
    for (int i = 0; i < NB; ++i) {
      const Fp2 d = fp2_dbl(fp2_dbl(s[i].g2));
      zero |= fp2_is_zero(d);
      run = i ? fp2_mul(run, d) : d;
      pre[i] = run;
    }
    if (!zero) {
      Fp2 inv = fp2_inv(run);  // 1 / (d_0 ... d_5)
      Fp12 acc = fp12_one();
#pragma unroll
      for (int i = NB - 1; i >= 0; --i) {
        const Fp2 inv_i = i ? fp2_mul(inv, pre[i - 1]) : inv;
        if (i) inv = fp2_mul(inv, fp2_dbl(fp2_dbl(s[i].g2)));
        const Fp12 e = cyc_decompress(s[i], inv_i);
        acc = (i == NB - 1) ? e : fp12_mul(acc, e);
      }
      return fp12_conj(acc);
    }
  }
#endif
  Fp12 acc = a;
  for (int b = 62; b >= 0; --b) {
    acc = fp12_cyc_sqr(acc);
    if ((Z_ABS >> b) & 1) acc = fp12_mul(acc, a);
  }
  return fp12_conj(acc);
}

DG12 Fp12 final_exp_cubed(const Fp12& f) {
  Fp12 f1 = fp12_mul(fp12_conj(f), fp12_inv(f));      // f^(p^6 - 1)
  Fp12 f2 = fp12_mul(fp12_frob(fp12_frob(f1)), f1);   // ^(p^2 + 1)
  Fp12 t0 = fp12_mul(cyc_exp_z(f2), fp12_conj(f2));   // f2^(z-1)
  Fp12 t1 = fp12_mul(cyc_exp_z(t0), fp12_conj(t0));   // f2^((z-1)^2)
  Fp12 a = fp12_mul(cyc_exp_z(t1), fp12_frob(t1));    // ^(z+p)
  Fp12 b = fp12_mul(cyc_exp_z(cyc_exp_z(a)), fp12_frob(fp12_frob(a)));
  b = fp12_mul(b, fp12_conj(a));                      // ^(z^2 + p^2 - 1)
  Fp12 c = fp12_mul(fp12_sqr(f2), f2);                // f2^3
  return fp12_mul(b, c);
}

}  // namespace dg
