// Recover as one multi-scalar multiplication per round (A6: kyber tbls.Recover at beacon/beacon.go:488 ->
// share.RecoverCommit; north_star: "Lagrange-in-the-exponent Recover as a ... multi-scalar multiplication").
//
//   sigma_r = sum_j lambda_j S_{r,j}            (t selected shares, lambda_j = prod_{m != j} x_m / (x_m - x_j))
//
// Every lambda_j < r is split into base-|z| digits (psi acts on G2 as [z], z = -|z|, r < |z|^4):
//   lambda_j = d0 + d1 |z| + d2 |z|^2 + d3 |z|^3   ->   [lambda_j]P = [d0]P - [d1]psi(P) + [d2]psi^2(P) - [d3]psi^3(P)
// so sigma_r = A0 - psi(A1) + psi^2(A2) - psi^3(A3) with A_i = sum_j [d_i(lambda_j)] S_{r,j}: four MSMs of t points
// with 64-bit scalars, one lane each, sharing ONE 64-doubling chain over all t points (Straus) instead of the
// t separate chains of t scalar multiplications (round 2).  The scalars are width-5 signed digits (wNAF: odd
// digits in [-15, 15], at most one non-zero in any 5 consecutive positions, ~11 per 64-bit digit), added from a
// table of the odd multiples 1P, 3P, ..., 15P of every share.
//
// Rounds are grouped in blocks of 64 (one wave).  A block whose OK rounds all selected the same index set --
// every round of a valid chain -- shares lambda, so its digit schedule (the ordered list of additions and
// doublings) is one wave-uniform list read with scalar loads: no divergence, no per-lane scalar.  Work per
// round: the tables (1 tangent + 7 chord affine additions per share, the denominators of each level inverted
// together over the whole batch: ~15 Fp products per addition), 4 x 64 doublings and ~11 t x 4 mixed additions,
// against 64 doublings + ~86 mixed additions PER SHARE before.
//   k_rc_blocks    per block: uniform?  first OK round (the block's lambda source)
//   k_rc_digits    per uniform block: lambda (one Fr inversion for all t), base-|z| digits, wNAF schedules
//   k_rc_tab_den / batch inversion / k_rc_tab_add     per level: the odd-multiple tables, affine (SoA in HBM)
//   k_rc_straus    lane (component i, round): A_i by the block's schedule, running point in LDS
//   k_rc_combine   per round: sigma = A0 - psi(A1) + psi^2(A2) - psi^3(A3)
// Blocks whose rounds selected different index sets (corrupted shares, C5) take the divergent-round form below
// (k_rs_*: one sign-aligned joint MSM per round, regular control flow whatever each lane's scalars).
#pragma once
// included from kernels.h (uses the G2AStore / G2JStore layouts, the Fr helpers and DG_ST_OK_ defined there)

#if !defined(__HIP__)
struct uint4 {  // the HIP vector type, for the host builds of this header (tests/native, tools/opcount)
  uint32_t x, y, z, w;
};
#endif

namespace dg {

constexpr uint32_t RC_W = 5;                                       // signed-digit width
constexpr uint32_t RC_TAB = 1u << (RC_W - 2);                      // 8 odd multiples per share
constexpr uint32_t RC_BLK = 64;                                    // rounds per block (one wave)
constexpr uint32_t RC_NAF = 65;                                    // digit positions of a 64-bit scalar
constexpr uint32_t RC_EV_PER_SHARE = (RC_NAF + RC_W - 1) / RC_W;   // at most 13 non-zero digits per scalar
constexpr uint32_t RC_Q = 12;                                      // uint4 words of one affine table entry

// schedule event: bits 0..15 share j, 16..18 table entry e (the multiple 2e + 1), 19 subtract, 20..27 doublings
// to run before this addition
DGI uint32_t rc_event(uint32_t j, uint32_t e, uint32_t neg, uint32_t dbl) { return j | e << 16 | neg << 19 | dbl << 20; }
DGI uint32_t rc_ev_j(uint32_t v) { return v & 0xffffu; }
DGI uint32_t rc_ev_e(uint32_t v) { return (v >> 16) & 7u; }
DGI bool rc_ev_neg(uint32_t v) { return (v >> 19) & 1u; }
DGI uint32_t rc_ev_dbl(uint32_t v) { return v >> 20; }

// width-RC_W non-adjacent form of a 64-bit scalar, positions 0..64 (65-bit arithmetic for the carry)
DGI void rc_wnaf(uint64_t d, int8_t* naf) {
  uint64_t lo = d, hi = 0;
  for (uint32_t b = 0; b < RC_NAF; ++b) {
    int z = 0;
    if (lo & 1u) {
      const int m = (int)(lo & ((1u << RC_W) - 1));
      z = m >= (1 << (RC_W - 1)) ? m - (1 << RC_W) : m;
      if (z > 0) {
        lo -= (uint64_t)z;  // lo mod 2^w = z: no borrow
      } else {
        const uint64_t s = lo + (uint64_t)(-z);
        hi += s < lo ? 1u : 0u;
        lo = s;
      }
    }
    naf[b] = (int8_t)z;
    lo = (lo >> 1) | (hi << 63);
    hi >>= 1;
  }
}

// The schedule of sum_j [d_j] P_j from the signed digits naf[j * RC_NAF + b] (Horner over the positions, top down;
// within a position by share): events ev[0..n), and `tail` doublings after the last one.  (k_rc_digits builds
// the same list with one lane per share and ballots.)
DGI uint32_t rc_schedule_naf(const int8_t* naf, uint32_t t, uint32_t* ev, uint32_t& tail) {
  uint32_t n = 0;
  int last = -1;
  for (int b = (int)RC_NAF - 1; b >= 0; --b)
    for (uint32_t j = 0; j < t; ++j) {
      const int z = naf[(size_t)RC_NAF * j + b];
      if (!z) continue;
      const uint32_t a = (uint32_t)(z < 0 ? -z : z);
      ev[n++] = rc_event(j, (a - 1) / 2, z < 0 ? 1u : 0u, last < 0 ? 0u : (uint32_t)(last - b));
      last = b;
    }
  tail = last < 0 ? 0u : (uint32_t)last;
  return n;
}

// (r - 1) / 2, little-endian limbs
DG_CONST uint32_t FR_HALF[8] = {0x80000000u, 0x7fffffffu, 0x7fff2dffu, 0xa9ded201u,
                                0x04d0ec02u, 0x199cec04u, 0x94cebea4u, 0x39f6d3a9u};
// Signed scalar: a plain k > (r - 1) / 2 is replaced by r - k and the share's point negated ([k]P = [r - k](-P)).
// For random k no gain; Lagrange coefficients of a run of consecutive indices are binomials +-C(t, j) (x_m = 1..t),
// whose negative half is r - C: as r - k they are small, and their digits d1..d3 vanish.  Returns the negation.
DGI bool rc_signed(Fr& k) {
  uint32_t br = 0;
  for (int i = 0; i < 8; ++i) (void)subb32(FR_HALF[i], k.l[i], br, &br);
  if (!br) return false;  // k <= (r - 1) / 2
  Fr z;
  for (int i = 0; i < 8; ++i) z.l[i] = 0;
  k = fr_sub(z, k);  // r - k (plain in, plain out: the subtraction is representation-free)
  return true;
}

// lambda_j (plain, 8 little-endian limbs) for j < t over the interpolation points x_m = idx[m] + 1 (kyber
// lagrangeBasis at 0), all t with one Fr inversion: den_j = x_j prod_{m != j} (x_m - x_j), inverted together
// (Montgomery's trick; `pre` holds the prefix products), lambda_j = (prod_m x_m) / den_j.
DGI void rc_lambdas(const uint32_t* idx, uint32_t t, Fr* lam, Fr* pre) {
  Fr num = fr_const(FR_ONE);
  for (uint32_t j = 0; j < t; ++j) {
    const Fr xj = fr_from_u32(idx[j] + 1);
    num = fr_mul(num, xj);
    Fr den = xj;
    for (uint32_t m = 0; m < t; ++m)
      if (m != j) den = fr_mul(den, fr_sub(fr_from_u32(idx[m] + 1), xj));
    lam[j] = den;
  }
  Fr acc = fr_const(FR_ONE);
  for (uint32_t j = 0; j < t; ++j) {
    pre[j] = acc;
    acc = fr_mul(acc, lam[j]);
  }
  Fr inv = fr_inv(acc);
  for (uint32_t j = t; j-- > 0;) {
    const Fr dj = lam[j];
    lam[j] = fr_to_plain(fr_mul(num, fr_mul(inv, pre[j])));  // 1 / den_j = inv(all) * prefix(j)
    inv = fr_mul(inv, dj);
  }
}

// base-|z| digits of a plain scalar k < r: d[0..3] (g2_mul_u256_psi's split)
DGI void rc_psi_digits(const Fr& k, uint64_t* d) {
  uint32_t q[8];
  for (int w = 0; w < 8; ++w) q[w] = k.l[w];
  d[0] = u256_divmod_u64(q, Z_ABS);
  d[1] = u256_divmod_u64(q, Z_ABS);
  d[2] = u256_divmod_u64(q, Z_ABS);
  d[3] = (uint64_t)q[1] << 32 | q[0];
}

// sigma = A0 - psi(A1) + psi^2(A2) - psi^3(A3), Horner in psi: psi(psi(psi(-A3) + A2) - A1) + A0
DGI G2J rc_combine(const G2J& a0, const G2J& a1, const G2J& a2, const G2J& a3) {
  G2J s = g2_psi(jac_neg(a3));
  s = g2_psi(jac_add(s, a2));
  s = g2_psi(jac_add(s, jac_neg(a1)));
  return jac_add(s, a0);
}

// SoA table access: one affine point as RC_Q uint4 words, word q at base[q * stride]
DGI void rc_ld(const uint4* base, size_t stride, Fp2& x, Fp2& y) {
  uint32_t w[48];
#pragma unroll
  for (uint32_t q = 0; q < RC_Q; ++q) {
    const uint4 v = base[q * stride];
    w[4 * q] = v.x;
    w[4 * q + 1] = v.y;
    w[4 * q + 2] = v.z;
    w[4 * q + 3] = v.w;
  }
#pragma unroll
  for (int i = 0; i < 12; ++i) {
    x.c0.l[i] = w[i];
    x.c1.l[i] = w[12 + i];
    y.c0.l[i] = w[24 + i];
    y.c1.l[i] = w[36 + i];
  }
}
DGI void rc_st(uint4* base, size_t stride, const Fp2& x, const Fp2& y) {
  uint32_t w[48];
#pragma unroll
  for (int i = 0; i < 12; ++i) {
    w[i] = x.c0.l[i];
    w[12 + i] = x.c1.l[i];
    w[24 + i] = y.c0.l[i];
    w[36 + i] = y.c1.l[i];
  }
#pragma unroll
  for (uint32_t q = 0; q < RC_Q; ++q) base[q * stride] = uint4{w[4 * q], w[4 * q + 1], w[4 * q + 2], w[4 * q + 3]};
}

#if defined(__HIP__) && DG_TU_LIB
// one wave per block of 64 rounds: uni[b] = 1 if every OK round of the block selected the same index set,
// ref[b] = the first OK round (~0u: the block has none)
DG_KERNEL void __launch_bounds__(64) k_rc_blocks(uint32_t R, uint32_t t, const uint32_t* selidx, const uint8_t* rst,
                                                 uint8_t* uni, uint32_t* ref) {
  const uint32_t b = blockIdx.x, r = b * RC_BLK + threadIdx.x;
  const bool ok = r < R && rst[r] == DG_ST_OK_;
  const uint64_t okm = __ballot(ok);
  if (okm == 0) {
    if (threadIdx.x == 0) {
      uni[b] = 1;
      ref[b] = ~0u;
    }
    return;
  }
  const int lead = __ffsll((unsigned long long)okm) - 1;
  bool same = true;
  for (uint32_t j = 0; j < t; ++j) {
    const uint32_t v = ok ? selidx[(size_t)r * t + j] : 0u;
    same = same && (!ok || v == (uint32_t)__shfl((int)v, lead));
  }
  const bool all = __all(same);
  if (threadIdx.x == 0) {
    uni[b] = all ? 1 : 0;
    ref[b] = b * RC_BLK + (uint32_t)lead;
  }
}

// One 64-lane workgroup per uniform block u (ub[u]), lanes over the shares j (t > 64: in chunks of 64): lambda_j
// of the block's reference round (each lane inverts its own denominator), signed (rc_signed), its base-|z| digits
// and their width-5 signed digits (naf: per (u, component, j) RC_NAF bytes of scratch, negated for a negated
// share); then per component the schedule, position-major and by share within a position, by one ballot per
// (position, chunk): ev[(u * 4 + i) * maxev ..], hdr[(u * 4 + i) * 2 + {0, 1}] = (events, tail doublings).
DG_KERNEL void __launch_bounds__(64) k_rc_digits(uint32_t U, uint32_t t, uint32_t maxev, const uint32_t* ub,
                                                 const uint32_t* ref, const uint32_t* selidx, int8_t* naf, uint32_t* ev,
                                                 uint32_t* hdr) {
  const uint32_t u = blockIdx.x, lane = threadIdx.x;
  if (u >= U) return;
  const uint32_t* idx = selidx + (size_t)ref[ub[u]] * t;
  Fr num = fr_const(FR_ONE);
  for (uint32_t m = 0; m < t; ++m) num = fr_mul(num, fr_from_u32(idx[m] + 1));
  for (uint32_t j = lane; j < t; j += RC_BLK) {
    const Fr xj = fr_from_u32(idx[j] + 1);
    Fr den = xj;
    for (uint32_t m = 0; m < t; ++m)
      if (m != j) den = fr_mul(den, fr_sub(fr_from_u32(idx[m] + 1), xj));
    Fr lam = fr_to_plain(fr_mul(num, fr_inv(den)));
    const bool neg = rc_signed(lam);
    uint64_t d[4];
    rc_psi_digits(lam, d);
    for (uint32_t i = 0; i < 4; ++i) {
      int8_t* z = naf + (((size_t)u * 4 + i) * t + j) * RC_NAF;
      rc_wnaf(d[i], z);
      if (neg)
        for (uint32_t b = 0; b < RC_NAF; ++b) z[b] = (int8_t)-z[b];
    }
  }
  __syncthreads();  // (the naf bytes are read back by other lanes: global memory, same workgroup)
  __threadfence_block();
  const uint64_t below = (1ull << lane) - 1;
  for (uint32_t i = 0; i < 4; ++i) {
    const int8_t* zi = naf + ((size_t)u * 4 + i) * t * RC_NAF;
    uint32_t* e = ev + ((size_t)u * 4 + i) * maxev;
    uint32_t n = 0;
    int last = -1;
    for (int b = (int)RC_NAF - 1; b >= 0; --b) {
      bool first = true;  // the first event at this position carries the doublings since the previous one
      for (uint32_t c = 0; c < t; c += RC_BLK) {
        const uint32_t j = c + lane;
        const int z = j < t ? zi[(size_t)j * RC_NAF + b] : 0;
        const uint64_t mask = __ballot(z != 0);
        if (!mask) continue;
        if (z) {
          const uint32_t pos = n + (uint32_t)__popcll(mask & below);
          const bool lead = first && (mask & below) == 0;
          const uint32_t a = (uint32_t)(z < 0 ? -z : z);
          e[pos] = rc_event(j, (a - 1) / 2, z < 0 ? 1u : 0u, lead && last >= 0 ? (uint32_t)(last - b) : 0u);
        }
        n += (uint32_t)__popcll(mask);
        first = false;
        last = b;
      }
    }
    if (lane == 0) {
      hdr[((size_t)u * 4 + i) * 2] = n;
      hdr[((size_t)u * 4 + i) * 2 + 1] = last < 0 ? 0u : (uint32_t)last;
    }
  }
}

// per round r of a uniform block: sigma = A0 - psi(A1) + psi^2(A2) - psi^3(A3) into out[r] (A: nsplit x 4 x Ru, the
// share subsets' parts of each A_i summed first; rounds in uniform-block order); rounds without status OK are left
// alone (k_compress_g2 writes zeros for them)
DG_KERNEL void __launch_bounds__(128, DG_BULK_WAVES) k_rc_combine(uint32_t R, uint32_t Ru, const uint32_t* ub,
                                                                  const uint8_t* rst, const G2JStore* A, G2JStore* out,
                                                                  uint32_t nsplit) {
  const uint32_t u = blockIdx.x * blockDim.x + threadIdx.x;
  if (u >= Ru) return;
  const uint32_t r = ub[u / RC_BLK] * RC_BLK + u % RC_BLK;
  if (r >= R || rst[r] != DG_ST_OK_) return;
  auto part = [&](uint32_t i) {
    G2J a = load_g2j(A[(size_t)i * Ru + u]);
#pragma unroll 1
    for (uint32_t s = 1; s < nsplit; ++s) a = jac_add(a, load_g2j(A[((size_t)s * 4 + i) * Ru + u]));
    return a;
  };
  store_g2j(out[r], rc_combine(part(0), part(1), part(2), part(3)));
}
#endif

#if defined(__HIP__) && DG_TU_HOT
// The tables, one level per launch pair with a batch inversion between them.  Lane g < t * Ru: share j = g / Ru
// of uniform round u = g % Ru.  Level 0: T[0] = P = S of the share, D = 2P (tangent); level l = 1..7:
// T[l] = T[l-1] + D (chord).  P in G2 has order r, so (2l - 1)P != +-2P: no exceptional pair; an identity share
// (possible only for an identity key) is flagged in pinf and skipped everywhere.
DGI bool rc_lane(uint32_t g, uint32_t t, uint32_t R, uint32_t Ru, const uint32_t* ub, const uint8_t* rst,
                 uint32_t& j, uint32_t& u, uint32_t& r) {
  if (g >= t * Ru) return false;
  j = g / Ru;
  u = g % Ru;
  r = ub[u / RC_BLK] * RC_BLK + u % RC_BLK;
  return r < R && rst[r] == DG_ST_OK_;
}
DG_KERNEL void __launch_bounds__(128) k_rc_tab_den(uint32_t l, uint32_t R, uint32_t Ru, uint32_t k, uint32_t t,
                                                   const uint32_t* ub, const uint8_t* rst, const uint32_t* sel,
                                                   const G2AStore* S, const uint4* T4, const uint4* D4, uint8_t* pinf,
                                                   Fp* den) {
  const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= t * Ru) return;
  uint32_t j, u, r;
  Fp n = fp_one();
  if (rc_lane(g, t, R, Ru, ub, rst, j, u, r)) {
    if (l == 0) {
      const G2AStore& p = S[(size_t)r * k + sel[(size_t)r * t + j]];
      pinf[g] = p.inf ? 1 : 0;
      if (!p.inf) n = fp2_norm(fp2_dbl(p.y));
    } else if (!pinf[g]) {
      Fp2 tx, ty, dx, dy;
      rc_ld(T4 + ((size_t)j * RC_TAB + (l - 1)) * RC_Q * Ru + u, Ru, tx, ty);
      rc_ld(D4 + (size_t)j * RC_Q * Ru + u, Ru, dx, dy);
      n = fp2_norm(fp2_sub(dx, tx));
    }
  }
  den[g] = n;
}
DG_KERNEL void __launch_bounds__(128, DG_HOT_WAVES) k_rc_tab_add(uint32_t l, uint32_t R, uint32_t Ru, uint32_t k, uint32_t t,
                                                                 const uint32_t* ub, const uint8_t* rst,
                                                                 const uint32_t* sel, const G2AStore* S, uint4* T4,
                                                                 uint4* D4, const uint8_t* pinf, const Fp* ninv) {
  const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t j, u, r;
  if (!rc_lane(g, t, R, Ru, ub, rst, j, u, r) || pinf[g]) return;
  if (l == 0) {
    const G2A p = load_g2a(S[(size_t)r * k + sel[(size_t)r * t + j]]);
    rc_st(T4 + (size_t)j * RC_TAB * RC_Q * Ru + u, Ru, p.x, p.y);
    const G2A d = g2_aff_sum(p, p, 2, ninv[g]);
    rc_st(D4 + (size_t)j * RC_Q * Ru + u, Ru, d.x, d.y);
  } else {
    G2A a{}, d{};
    rc_ld(T4 + ((size_t)j * RC_TAB + (l - 1)) * RC_Q * Ru + u, Ru, a.x, a.y);
    rc_ld(D4 + (size_t)j * RC_Q * Ru + u, Ru, d.x, d.y);
    a.inf = d.inf = false;
    const G2A s = g2_aff_sum(a, d, 1, ninv[g]);
    rc_st(T4 + ((size_t)j * RC_TAB + l) * RC_Q * Ru + u, Ru, s.x, s.y);
  }
}

// One 64-lane workgroup per (component i, uniform block, share subset s < nsplit): lane = round of the block; the
// part of A_i from the shares j = s mod nsplit by the block's schedule (wave-uniform: scalar loads, uniform branches;
// every subset runs the whole doubling chain), the running point in LDS (g2_madd_lds / g2_dbl_lds: the register file
// holds one table entry and one formula's temporaries); A[(s 4 + i) Ru + u], summed by k_rc_combine.  nsplit > 1 when
// the blocks are too few to fill the chip (the live round: one block, whose ~430 dependent point operations took 7 ms
// in one lane; drand_gpu.hip recover_msm)
DG_KERNEL void __launch_bounds__(64, DG_TERMS_WAVES) k_rc_straus(uint32_t R, uint32_t Ru, uint32_t maxev, const uint32_t* ub,
                                                                 const uint8_t* rst, const uint32_t* ev,
                                                                 const uint32_t* hdr, const uint4* T4,
                                                                 const uint8_t* pinf, G2JStore* A, uint32_t nsplit) {
  const uint32_t U = Ru / RC_BLK, s = blockIdx.x % nsplit, w = blockIdx.x / nsplit, i = w / U, ubk = w % U;  // uniform
  const uint32_t u = ubk * RC_BLK + threadIdx.x, r = ub[ubk] * RC_BLK + threadIdx.x;
  const bool live = r < R && rst[r] == DG_ST_OK_;
  const uint32_t* e = ev + ((size_t)ubk * 4 + i) * maxev;
  const uint32_t n = hdr[((size_t)ubk * 4 + i) * 2], tail = hdr[((size_t)ubk * 4 + i) * 2 + 1];
  __shared__ G2JStore s_acc[RC_BLK];
  G2JStore& acc = s_acc[threadIdx.x];
  acc.x = fp2_zero();
  acc.y = fp2_zero();
  acc.z = fp2_zero();
  for (uint32_t q = 0; q < n; ++q) {
    const uint32_t v = e[q];
    for (uint32_t d = rc_ev_dbl(v); d > 0; --d) g2_dbl_lds(acc);
    const uint32_t j = rc_ev_j(v);
    if (live && j % nsplit == s && !pinf[(size_t)j * Ru + u]) {
      Fp2 x, y;
      rc_ld(T4 + ((size_t)j * RC_TAB + rc_ev_e(v)) * RC_Q * Ru + u, Ru, x, y);
      g2_madd_lds(acc, x, rc_ev_neg(v) ? fp2_neg(y) : y);
    }
  }
  for (uint32_t d = tail; d > 0; --d) g2_dbl_lds(acc);
  if (live) A[((size_t)s * 4 + i) * Ru + u] = acc;
}
#elif defined(__HIP__)
DG_KERNEL void __launch_bounds__(128) k_rc_tab_den(uint32_t l, uint32_t R, uint32_t Ru, uint32_t k, uint32_t t,
                                                   const uint32_t* ub, const uint8_t* rst, const uint32_t* sel,
                                                   const G2AStore* S, const uint4* T4, const uint4* D4, uint8_t* pinf,
                                                   Fp* den);
DG_KERNEL void __launch_bounds__(128, DG_HOT_WAVES) k_rc_tab_add(uint32_t l, uint32_t R, uint32_t Ru, uint32_t k, uint32_t t,
                                                                 const uint32_t* ub, const uint8_t* rst,
                                                                 const uint32_t* sel, const G2AStore* S, uint4* T4,
                                                                 uint4* D4, const uint8_t* pinf, const Fp* ninv);
DG_KERNEL void __launch_bounds__(64, DG_TERMS_WAVES) k_rc_straus(uint32_t R, uint32_t Ru, uint32_t maxev, const uint32_t* ub,
                                                                 const uint8_t* rst, const uint32_t* ev,
                                                                 const uint32_t* hdr, const uint4* T4,
                                                                 const uint8_t* pinf, G2JStore* A, uint32_t nsplit);
#endif

// ---------------------------------------------------------------------------------------------------
// Divergent rounds (blocks whose rounds selected different index sets: corrupted shares, C5): one joint MSM per
// round in the sign-aligned column form (GLV-SAC, curve.h g2_mul_u256_psi_sac) -- every lane runs the same
// column loop whatever its scalars, so lanes holding different rounds never diverge.  Per share j, with its
// psi digits d0..d3 (d0 made odd, corrected by one final subtraction of P_j), column c adds s_c T_j[u_c],
// T_j[u] = P0 + u1 P1 + u2 P2 + u3 P3 (P0 = P, P1 = -psi(P), P2 = psi^2(P), P3 = -psi^3(P)): 65 columns.  A lane
// takes RS_G shares of one round and shares ONE doubling per column among them (the round-2 per-term form paid 65
// doublings per share); the RS_G-share partial sums of a round are added at the end.  The tables are affine,
// built in three batched levels (T1, T2, T4 = P0 + P1, P0 + P2, P0 + P3; T3, T5, T6 = T1 + P2, T1 + P3, T2 + P3;
// T7 = T3 + P3) with the denominators of each level inverted together.  P_i are [|z|^i]P up to sign with
// 1 + |z| + |z|^2 + |z|^3 < r, so for P != O no table addition is exceptional.
//   k_rs_digits    lane (share, round): lambda_j, psi digits, sign-aligned recoding (RsDigits)
//   k_rs_tab_den / batch inversion / k_rs_tab_add     three levels of the 8-entry tables
//   k_rs_sac       lane (share group, round): the group's joint column loop, running point in LDS
//   k_rs_combine   per round: the sum of its group partial sums
constexpr uint32_t RS_G = 8;  // shares per lane (default; DG_RS_G)
constexpr uint32_t RS_DIG_NT = 256;  // k_rs_digits' workgroup: one Fr inversion per 256 coefficients

// sign-aligned recoding of one share's psi digits (g2_mul_u256_psi_sac): bit c of sgn set = +T in column c
// (c < 64; column 64 is always +), um[i] bit c = u_{i+1, c}, top = the column-64 entry, even: d0 was even (add
// 1, subtract P at the end)
struct RsDigits {
  uint64_t sgn, um[3];
  uint32_t top, even;
};
DGI RsDigits rs_recode(const uint64_t (&d)[4]) {
  RsDigits o;
  o.even = (d[0] & 1) == 0 ? 1u : 0u;
  const uint64_t k0 = d[0] + (o.even ? 1u : 0u);
  o.sgn = k0 >> 1;
  o.top = 0;
  for (int i = 0; i < 3; ++i) {
    uint64_t a = d[i + 1], m = 0;
    for (int j = 0; j < 64; ++j) {
      const uint64_t bit = a & 1u;
      m |= bit << j;
      a = (a >> 1) + (bit & ~(o.sgn >> j) & 1u);
    }
    o.um[i] = m;
    o.top |= (uint32_t)a << i;
  }
  return o;
}
// P0..P3 of a share (the same signs as g2_mul_u256_psi_sac: P1 = -psi(P), P2 = psi^2(P) = (w x, -y),
// P3 = -psi^3(P) = (w psi(P).x, psi(P).y))
DGI void rs_points(const G2A& p, Fp2 (&px)[4], Fp2 (&py)[4]) {
  Fp2 qx = p.x, qy = p.y;
  g2_psi_aff(qx, qy);
  const Fp w = fp_const(PSI2_W);
  px[0] = p.x;
  py[0] = p.y;
  px[1] = qx;
  py[1] = fp2_neg(qy);
  px[2] = fp2_mul_fp(p.x, w);
  py[2] = fp2_neg(p.y);
  px[3] = fp2_mul_fp(qx, w);
  py[3] = qy;
}
// table level l (0..2), element e (0..2): the pair (a index, b point) it adds and the entry it writes
//   l0: T1 = T0 + P1, T2 = T0 + P2, T4 = T0 + P3;  l1: T3 = T1 + P2, T5 = T1 + P3, T6 = T2 + P3;  l2: T7 = T3 + P3
DGI bool rs_level(uint32_t l, uint32_t e, uint32_t& src, uint32_t& pb, uint32_t& dst) {
  constexpr uint8_t S[3][3] = {{0, 0, 0}, {1, 1, 2}, {3, 0, 0}};
  constexpr uint8_t B[3][3] = {{1, 2, 3}, {2, 3, 3}, {3, 0, 0}};
  constexpr uint8_t D[3][3] = {{1, 2, 4}, {3, 5, 6}, {7, 0, 0}};
  if (l == 2 && e > 0) return false;
  src = S[l][e];
  pb = B[l][e];
  dst = D[l][e];
  return true;
}

#if defined(__HIP__) && DG_TU_LIB
// 1 / v for the NT threads of a workgroup by Montgomery's trick: per wave the inclusive prefix and suffix products
// (shuffle scans, 12 Fr products a lane), the wave totals inverted together by thread 0 (ONE Fr inversion per
// workgroup instead of one per lane: a lane's inversion is ~300 products and a wave pays it whether 1 or 64 lanes
// need it), then 1 / v_i = (prod_{k < i} v_k)(prod_{k > i} v_k) / total_w.  v != 0; every thread calls it.
template <uint32_t NT>
DGI Fr fr_inv_block(const Fr& v) {
  constexpr uint32_t NW = NT / 64;
  __shared__ Fr s_w[NW];
  const uint32_t lane = threadIdx.x & 63u, w = threadIdx.x >> 6;
  Fr pre = v, suf = v;
#pragma unroll 1
  for (uint32_t d = 1; d < 64; d <<= 1) {
    Fr a, b;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      a.l[i] = __shfl_up(pre.l[i], d, 64);
      b.l[i] = __shfl_down(suf.l[i], d, 64);
    }
    if (lane >= d) pre = fr_mul_in(pre, a);
    if (lane + d < 64) suf = fr_mul_in(suf, b);
  }
  Fr ep, es;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    ep.l[i] = __shfl_up(pre.l[i], 1, 64);
    es.l[i] = __shfl_down(suf.l[i], 1, 64);
  }
  if (lane == 0) ep = fr_const(FR_ONE);
  if (lane == 63) {
    es = fr_const(FR_ONE);
    s_w[w] = pre;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    Fr p[NW], acc = fr_const(FR_ONE);
#pragma unroll
    for (uint32_t k = 0; k < NW; ++k) {
      p[k] = acc;
      acc = fr_mul_in(acc, s_w[k]);
    }
    Fr inv = fr_inv_in(acc);
#pragma unroll
    for (uint32_t k = NW; k-- > 0;) {
      const Fr tw = s_w[k];
      s_w[k] = fr_mul_in(inv, p[k]);
      inv = fr_mul_in(inv, tw);
    }
  }
  __syncthreads();
  return fr_mul_in(fr_mul_in(ep, es), s_w[w]);
}

// lane g < t * Rn: share j = g % t of divergent round u = g / t (round nl[u]; a wave reads one or two rounds' index
// rows); lambda_j of the round's own selected set (lagrange_nd, the workgroup's shared inversion), its psi digits
// and their sign-aligned recoding, dig[j * Rn + u]
DG_KERNEL void __launch_bounds__(RS_DIG_NT) k_rs_digits(uint32_t R, uint32_t Rn, uint32_t t, const uint32_t* nl,
                                                        const uint32_t* selidx, const uint8_t* rst, RsDigits* dig) {
  const uint32_t g = blockIdx.x * RS_DIG_NT + threadIdx.x;
  const uint32_t u = g / t, j = g % t;
  const uint32_t r = g < t * Rn ? nl[u] : R;
  const bool live = r < R && rst[r] == DG_ST_OK_;
  Fr num, den = fr_const(FR_ONE);
  if (live) lagrange_nd(selidx + (size_t)r * t, t, j, num, den);
  uint32_t nz = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) nz |= den.l[i];
  const Fr dinv = fr_inv_block<RS_DIG_NT>(nz ? den : fr_const(FR_ONE));  // 0 (repeated index): lambda 0, as fr_inv
  if (!live) return;
  Fr lam = lagrange_finish(num, dinv);
  if (!nz)
#pragma unroll
    for (int i = 0; i < 8; ++i) lam.l[i] = 0;
  uint64_t d[4];
  rc_psi_digits(lam, d);
  dig[(size_t)j * Rn + u] = rs_recode(d);
}

// per divergent round u: sigma = the sum of its ngroups group partial sums (Aps[q * Rn + u]) into out[r]
DG_KERNEL void __launch_bounds__(128, DG_BULK_WAVES) k_rs_combine(uint32_t R, uint32_t Rn, uint32_t ngroups,
                                                                  const uint32_t* nl, const uint8_t* rst,
                                                                  const G2JStore* Aps, G2JStore* out) {
  const uint32_t u = blockIdx.x * blockDim.x + threadIdx.x;
  if (u >= Rn) return;
  const uint32_t r = nl[u];
  if (r >= R || rst[r] != DG_ST_OK_) return;
  G2J acc = load_g2j(Aps[u]);
  for (uint32_t q = 1; q < ngroups; ++q) acc = jac_add(acc, load_g2j(Aps[(size_t)q * Rn + u]));
  store_g2j(out[r], acc);
}
#endif

#if defined(__HIP__) && DG_TU_HOT
// table entry e of share j in divergent round u: a lane's eight entries are contiguous (8 x 192 B), so the column
// loop's data-dependent pick reads 192 consecutive bytes per lane (the round-4 layout, entry-major with the rounds
// innermost, coalesced only lanes that picked the same entry: ~8x the bytes fetched)
DGI const uint4* rs_entry(const uint4* T4, uint32_t j, uint32_t u, uint32_t e, uint32_t Rn) {
  return T4 + (((size_t)j * Rn + u) * 8 + e) * RC_Q;
}
DGI uint4* rs_entry(uint4* T4, uint32_t j, uint32_t u, uint32_t e, uint32_t Rn) {
  return T4 + (((size_t)j * Rn + u) * 8 + e) * RC_Q;
}
DGI bool rs_lane(uint32_t g, uint32_t t, uint32_t R, uint32_t Rn, const uint32_t* nl, const uint8_t* rst,
                 uint32_t& j, uint32_t& u, uint32_t& r) {
  if (g >= t * Rn) return false;
  j = g / Rn;
  u = g % Rn;
  r = nl[u];
  return r < R && rst[r] == DG_ST_OK_;
}
// lane g < 3 t Rn: element e = g / (t Rn) of level l for (share j, round u); pinf[j * Rn + u] is set at level 0
DG_KERNEL void __launch_bounds__(128) k_rs_tab_den(uint32_t l, uint32_t R, uint32_t Rn, uint32_t k, uint32_t t,
                                                   const uint32_t* nl, const uint8_t* rst, const uint32_t* sel,
                                                   const G2AStore* S, const uint4* T4, uint8_t* pinf, Fp* den) {
  const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x, n = t * Rn;
  if (g >= 3 * n) return;
  const uint32_t e = g / n;
  uint32_t j, u, r, src, pb, dst;
  Fp v = fp_one();
  if (rs_lane(g % n, t, R, Rn, nl, rst, j, u, r) && rs_level(l, e, src, pb, dst)) {
    const G2A p = load_g2a(S[(size_t)r * k + sel[(size_t)r * t + j]]);
    if (l == 0 && e == 0) pinf[g % n] = p.inf ? 1 : 0;
    if (!p.inf) {
      Fp2 px[4], py[4];
      rs_points(p, px, py);
      Fp2 ax = px[0], ay;
      if (src) rc_ld(rs_entry(T4, j, u, src, Rn), 1, ax, ay);
      v = fp2_norm(fp2_sub(px[pb], ax));
    }
  }
  den[g] = v;
}
DG_KERNEL void __launch_bounds__(128, DG_HOT_WAVES) k_rs_tab_add(uint32_t l, uint32_t R, uint32_t Rn, uint32_t k, uint32_t t,
                                                                 const uint32_t* nl, const uint8_t* rst,
                                                                 const uint32_t* sel, const G2AStore* S, uint4* T4,
                                                                 const uint8_t* pinf, const Fp* ninv) {
  const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x, n = t * Rn;
  if (g >= 3 * n) return;
  const uint32_t e = g / n;
  uint32_t j, u, r, src, pb, dst;
  if (!rs_lane(g % n, t, R, Rn, nl, rst, j, u, r) || !rs_level(l, e, src, pb, dst) || pinf[g % n]) return;
  const G2A p = load_g2a(S[(size_t)r * k + sel[(size_t)r * t + j]]);
  Fp2 px[4], py[4];
  rs_points(p, px, py);
  G2A a{px[0], py[0], false};
  if (src) rc_ld(rs_entry(T4, j, u, src, Rn), 1, a.x, a.y);
  else if (e == 0) rc_st(rs_entry(T4, j, u, 0, Rn), 1, px[0], py[0]);  // T0 = P0 (level 0, once)
  const G2A s = g2_aff_sum(a, G2A{px[pb], py[pb], false}, 1, ninv[g]);
  rc_st(rs_entry(T4, j, u, dst, Rn), 1, s.x, s.y);
}

// lane (share group q, divergent round u), grid RS lanes = ngroups * Rn padded to whole waves: the columns of
// its <= gs shares (RS_G unless DG_RS_G), one doubling per column, then the even-d0 corrections; Aps[q * Rn + u]
DG_KERNEL void __launch_bounds__(64, DG_TERMS_WAVES) k_rs_sac(uint32_t R, uint32_t Rn, uint32_t t, uint32_t ngroups,
                                                              uint32_t gs, const uint32_t* nl, const uint8_t* rst,
                                                              const RsDigits* dig, const uint4* T4,
                                                              const uint8_t* pinf, G2JStore* Aps) {
  const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t q = g / Rn, u = g % Rn;
  const bool live = q < ngroups && nl[u] < R && rst[nl[u]] == DG_ST_OK_;
  const uint32_t j0 = q * gs, j1 = j0 + gs < t ? j0 + gs : t;
  __shared__ G2JStore s_acc[64];
  G2JStore& acc = s_acc[threadIdx.x];
  acc.x = fp2_zero();
  acc.y = fp2_zero();
  acc.z = fp2_zero();
  if (!live) return;
  for (int c = 64; c >= 0; --c) {
    if (c < 64) g2_dbl_lds(acc);
    for (uint32_t j = j0; j < j1; ++j) {
      if (pinf[(size_t)j * Rn + u]) continue;
      const RsDigits& d = dig[(size_t)j * Rn + u];
      uint32_t e;
      bool pos;
      if (c == 64) {
        e = d.top;
        pos = true;
      } else {
        e = (uint32_t)((d.um[0] >> c) & 1u) | (uint32_t)((d.um[1] >> c) & 1u) << 1 | (uint32_t)((d.um[2] >> c) & 1u) << 2;
        pos = (d.sgn >> c) & 1u;
      }
      Fp2 x, y;
      rc_ld(rs_entry(T4, j, u, e, Rn), 1, x, y);
      g2_madd_lds(acc, x, pos ? y : fp2_neg(y));
    }
  }
  for (uint32_t j = j0; j < j1; ++j) {
    if (pinf[(size_t)j * Rn + u] || !dig[(size_t)j * Rn + u].even) continue;
    Fp2 x, y;
    rc_ld(rs_entry(T4, j, u, 0, Rn), 1, x, y);
    g2_madd_lds(acc, x, fp2_neg(y));
  }
  Aps[(size_t)q * Rn + u] = acc;
}
#elif defined(__HIP__)
DG_KERNEL void __launch_bounds__(128) k_rs_tab_den(uint32_t l, uint32_t R, uint32_t Rn, uint32_t k, uint32_t t,
                                                   const uint32_t* nl, const uint8_t* rst, const uint32_t* sel,
                                                   const G2AStore* S, const uint4* T4, uint8_t* pinf, Fp* den);
DG_KERNEL void __launch_bounds__(128, DG_HOT_WAVES) k_rs_tab_add(uint32_t l, uint32_t R, uint32_t Rn, uint32_t k, uint32_t t,
                                                                 const uint32_t* nl, const uint8_t* rst,
                                                                 const uint32_t* sel, const G2AStore* S, uint4* T4,
                                                                 const uint8_t* pinf, const Fp* ninv);
DG_KERNEL void __launch_bounds__(64, DG_TERMS_WAVES) k_rs_sac(uint32_t R, uint32_t Rn, uint32_t t, uint32_t ngroups,
                                                              uint32_t gs, const uint32_t* nl, const uint8_t* rst,
                                                              const RsDigits* dig, const uint4* T4,
                                                              const uint8_t* pinf, G2JStore* Aps);
#endif

}  // namespace dg
