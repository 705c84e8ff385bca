// Isolation of a failed single-key batch (VerifyBeacon / bls.Verify against one group key) by adaptive group tests
// ACROSS rounds, on the pairing-check pipeline of checks.h.
//
// kyber decides every beacon alone (beacon/chain.go:65-71, beacon/beacon.go:575: one VerifyRecovered per round).  The
// batch equation of a chain decides them all at once when it holds; when it fails (a bad round anywhere in the batch),
// the rounds must still get exact verdicts.  One pairing check per round would cost ~20 k Fp products each, ~4x the
// whole batch.  Instead, with X the group key and independent 64-bit weights rho_i bound to the batch (Fiat-Shamir seed
// of kernels.h k_digest_*):
//     e(X, h_eff(sum rho_i Q_i)) == e(g1, sum rho_i S_i)          (Q_i the uncleared hash of round i: h_eff is linear)
// holds for a set of valid rounds, and a set holding a bad round passes with probability <= 2^-63 (every S_i in G2 --
// the batch's windowed subgroup check, or k_xg_sub after it failed -- and E_i = x h(Q_i) - S_i != 0 vanishes in the
// weighted sum for at most one rho_i mod r).  Two levels, each one run of the pipeline with its checks listed on the
// device:
//     level 1  groups of qpg quads (4 qpg rounds; default 16)          -> a failed group lists its rounds
//     level 3  single rounds: e(X, h(Q_i)) == e(g1, S_i), kyber's bls.Verify verdict, exact
// (the numbering keeps the round-5 counters: a level 2 of quads between them measured slower, 2.8 against 3.3 M
// rounds/s, and is gone).  Every round of a passed group keeps its OK status (error <= 2^-63); every rejected round was
// rejected by its own exact check.  At 1% bad rounds a 100k-round batch takes ~6.3 k + ~15 k checks instead of 100 k.
//
//   k_xg_sub    (after a failed windowed subgroup check only) the G2 subgroup check of every decoded signature
//   k_xg_cand   the decoded rounds of a failed batch, compacted (nothing after a passed batch)
//   k_xq_sum    per quad and side: sum rho_i P_i (P = Q or S) by the four-point sign-aligned column form over an affine
//               8-entry table built in the lane (three levels of affine additions, one Fp inversion per level)
//   per level:  k_xg_prep (the check's sums; sigma side affine), k_xg_heff (h_eff of the hash side), k_xg_miller (both
//               pairs' Miller values, their lines computed in the lane), checks.h k_ck_easy .. k_ck_final (gated on
//               the level's device count), k_xg_verdict
// The launches are sized for the worst case (every round bad: every round a single check) and gated on the device
// counts, so the host enqueues the whole isolation without a round trip; after a passed batch every launch returns at
// once.  A check's workspace is ~5 KB (its state and Fp12 values: no line table), ~0.7 GB for a 131072-round segment
// (round 5 stored both pairs' lines, ~45 KB a check, ~6 GB a segment, per workspace set).
#pragma once

namespace dg {

constexpr uint64_t XR_TAG = 0x63726f7373726e64ull;  // "crossrnd": domain of the cross-round weights rho_i
constexpr uint32_t XR_QPG = 4;                       // quads per level-1 group (default; DG_XR_QPG, a test hook)
// device counters: [0] candidates, [1] level-1 checks, [2] unused, [3] level-3 checks (rounds)
constexpr uint32_t XR_NCNT = 4;

DGI uint64_t xr_rho(uint64_t seed, uint32_t i) { return rlc_coeff(seed ^ XR_TAG, i); }

// the uncleared hash Q_i (Jacobian; Z = 1 or 0 from k_h2c_p4b) in affine form, exactly for any Z
DGI G2A xr_q_aff(const G2JStore& s) {
  const G2J q = load_g2j(s);
  if (jac_is_inf(q)) return G2A{fp2_zero(), fp2_zero(), true};
  if (fp2_eq(q.z, fp2_one())) return G2A{q.x, q.y, false};
  return g2_to_aff(q);
}

// sum rho_m P_m over four points (any may be the identity, repeat or cancel) by the sign-aligned column form of
// curve.h jac_msm4_sac: T[u] = P0 + u1 P1 + u2 P2 + u3 P3 built in three levels of exact affine pair additions (curve.h
// g2_aff_kind / g2_aff_den / g2_aff_sum: chord, tangent, P + (-P), identity operands) with one Fp inversion per level
// (Montgomery's trick over its <= 3 norms), the table kept by putT / getT (HBM on the device), the 65 columns into the
// accumulator `acc` (an LDS slot on the device).  member(m): P_m.
template <class Member, class GetT, class PutT, class Slot>
DGI void xq_sum4(Member member, const uint64_t (&rho)[4], GetT getT, PutT putT, Slot& acc) {
  putT(0, member(0));
#pragma unroll 1
  for (uint32_t l = 0; l < 3; ++l) {
    const uint32_t ne = l == 2 ? 1u : 3u;
    uint32_t kind[3];
    Fp den[3];
#pragma unroll
    for (uint32_t e = 0; e < 3; ++e) {
      uint32_t src, pb, dst;
      den[e] = fp_one();
      kind[e] = 0;
      if (e >= ne || !rs_level(l, e, src, pb, dst)) continue;
      const G2A A = getT(src), B = member(pb);
      kind[e] = g2_aff_kind(A, B);
      den[e] = g2_aff_den(A, B, kind[e]);
    }
    // 1 / den[e] from one inversion of their product (every norm is non-zero: g2_aff_den gives 1 where none is needed)
    const Fp p01 = fp_mul(den[0], den[1]);
    const Fp ip = fp_inv(fp_mul(p01, den[2]));
    const Fp ip01 = fp_mul(ip, den[2]);
    const Fp inv[3] = {fp_mul(ip01, den[1]), fp_mul(ip01, den[0]), fp_mul(ip, p01)};
#pragma unroll
    for (uint32_t e = 0; e < 3; ++e) {
      uint32_t src, pb, dst;
      if (e >= ne || !rs_level(l, e, src, pb, dst)) continue;
      putT(dst, g2_aff_sum(getT(src), member(pb), kind[e], inv[e]));
    }
  }
  ck_sac_g2(rs_recode(rho), getT, acc);
}

#if defined(__HIP__)
#if DG_TU_CHECK == 6
// the G2 subgroup check of every decoded signature of items [i0, i0 + n) of a FAILED batch (flag[0] == 0) whose windowed
// check failed (flag[2] != 0): outside G2 is kyber's decode error.  With flag[2] == 0 every signature the batch summed is
// in G2 except with probability 2^-66 (msm.h) and the group tests need no per-item check.  Lane 0 clears the counters.
DG_KERNEL void __launch_bounds__(64, DG_CK_SUB_WAVES) k_xg_sub(uint32_t i0, uint32_t n, const uint32_t* flag,
                                                               const G2AStore* S, uint8_t* status, uint32_t* cnt) {
  DG_HI();
  const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  __shared__ G2JStore s_acc[64];
  if (g == 0)
#pragma unroll
    for (uint32_t c = 0; c < XR_NCNT; ++c) cnt[c] = 0;
  if (g >= n || flag[0] || !flag[2]) return;
  const uint32_t i = i0 + g;
  if (status[i] != DG_ST_OK_) return;
  const G2A s = load_g2a(S[i]);
  if (!s.inf && !ck_in_subgroup(s.x, s.y, s_acc[threadIdx.x])) status[i] = DG_ST_SIG_DECODE_;
}
// one check of `level` (1: group g of qpg quads, 3: round l3list[g] alone; gcnt: the launch's device count): HS[g] = its
// uncleared hash-side sum, st[g] = {a: the group key, b: the signature-side sum (affine), np bit 1}
DG_KERNEL void __launch_bounds__(64, DG_CK_WAVES2) k_xg_prep(uint32_t level, uint32_t G, const uint32_t* gcnt,
                                                             const uint32_t* cnt, uint32_t qpg, const uint32_t* l3list,
                                                             const G2JStore* QS, const G2JStore* Q, const G2AStore* S,
                                                             const G1AStore* keys, CkState* st, G2JStore* HS) {
  DG_HI();
  const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  __shared__ G2JStore s_h[64], s_s[64];
  if (ck_dead(g, G, gcnt)) return;
  CkState c{};
  G2A b;
  if (level == 3) {
    const uint32_t i = l3list[g];
    HS[g] = Q[i];
    b = load_g2a(S[i]);
    c.live[0] = i;
  } else {
    const uint32_t nq = (cnt[0] + 3) / 4;
    const uint32_t q0 = g * qpg, q1 = q0 + qpg < nq ? q0 + qpg : nq;
    G2JStore& h = s_h[threadIdx.x];
    G2JStore& s = s_s[threadIdx.x];
    h.x = h.y = h.z = fp2_zero();
    s.x = s.y = s.z = fp2_zero();
#pragma unroll 1
    for (uint32_t q = q0; q < q1; ++q) {
      g2_add_lds(h, load_g2j(QS[2 * (size_t)q]));
      g2_add_lds(s, load_g2j(QS[2 * (size_t)q + 1]));
    }
    HS[g] = h;
    b = g2_to_aff(load_g2j(s));
    c.live[0] = q0;
  }
  c.a = keys[0];
  store_g2a(c.b, b);
  c.round = g;
  c.np = b.inf ? 0u : 2u;
  c.n = c.nl = 1;
  st[g] = c;
}
// H = h_eff(HS[g]) in place, affine (z = 1; the identity z = 0), and np bit 0 when neither H nor a is the identity --
// a kernel of its own, so the cofactor clearing's registers do not add to the Miller loop's
DG_KERNEL void __launch_bounds__(64, DG_CK_WAVES) k_xg_heff(uint32_t G, const uint32_t* gcnt, G2JStore* HS, CkState* st) {
  DG_HI();
  const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  if (ck_dead(g, G, gcnt)) return;
  const G2A h = g2_to_aff(g2_clear_cofactor(load_g2j(HS[g])));
  store_g2j(HS[g], h.inf ? G2J{fp2_zero(), fp2_zero(), fp2_zero()} : G2J{h.x, h.y, fp2_one()});
  if (!h.inf && !st[g].a.inf) st[g].np |= 1u;
}
// The Miller value of one pair of check g, its lines computed in the lane (checks.h ck_miller1_fly): lanes [0, Gp) pair 0
// = (a, H) with H = HS[g] from k_xg_heff, lanes [Gp, 2 Gp) pair 1 = (-g1, b), Gp = G rounded up to whole waves, so the
// two chains run side by side; F[pair G + g] (k_ck_easy multiplies the two).  No line table: round 5 wrote both pairs'
// 68 lines to HBM (k_xg_lines, 2 x 19.6 KB per check) for k_ck_miller2 to read back.
DG_KERNEL void __launch_bounds__(64, DG_CK_WAVES) k_xg_miller(uint32_t G, const uint32_t* gcnt, const G2JStore* HS,
                                                              const CkState* st, Fp12* F) {
  DG_HI();
  const uint32_t Gp = (G + 63) & ~63u, lane = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t pair = lane >= Gp ? 1u : 0u, g = lane - pair * Gp;
  __shared__ G2JStore s_T[64];
  if (ck_dead(g, G, gcnt)) return;
  Fp12 f = fp12_one();
  if ((st[g].np >> pair) & 1) {
    // pair 1: b at P = -g1; pair 0: H at P = a
    const auto q = [&]() { return pair ? load_g2a(st[g].b) : G2A{HS[g].x, HS[g].y, false}; };
    const Fp px = pair ? fp_const(G1_GEN_X) : st[g].a.x, py = pair ? fp_const(G1_GEN_NEG_Y) : st[g].a.y;
    f = ck_miller1_fly(q, px, py, s_T[threadIdx.x]);
  }
  F[(size_t)pair * G + g] = f;
}
#else
DG_KERNEL void __launch_bounds__(64, DG_CK_WAVES) k_xg_miller(uint32_t G, const uint32_t* gcnt, const G2JStore* HS,
                                                              const CkState* st, Fp12* F);
DG_KERNEL void __launch_bounds__(64, DG_CK_WAVES) k_xg_heff(uint32_t G, const uint32_t* gcnt, G2JStore* HS, CkState* st);
DG_KERNEL void __launch_bounds__(64, DG_CK_SUB_WAVES) k_xg_sub(uint32_t i0, uint32_t n, const uint32_t* flag,
                                                               const G2AStore* S, uint8_t* status, uint32_t* cnt);
DG_KERNEL void __launch_bounds__(64, DG_CK_WAVES2) k_xg_prep(uint32_t level, uint32_t G, const uint32_t* gcnt,
                                                             const uint32_t* cnt, uint32_t qpg, const uint32_t* l3list,
                                                             const G2JStore* QS, const G2JStore* Q, const G2AStore* S,
                                                             const G1AStore* keys, CkState* st, G2JStore* HS);
#endif
#if DG_TU_CHECK == 5
// lane 2 q + side (side 0: the hashes Q, side 1: the signatures S) of quad q = candidates [4 q, 4 q + 4): QS[2 q + side] =
// sum rho_i P_i (xq_sum4; the table SoA at T4 / tinf with stride 2 nqmax).  Lane 0 sets the level-1 count from the
// candidate count: ceil(nq / qpg) groups.
DG_KERNEL void __launch_bounds__(64, DG_CK_WAVES2) k_xq_sum(uint32_t nqmax, uint32_t qpg, const uint64_t* seedp,
                                                            uint32_t* cnt, const uint32_t* cand, const G2JStore* Q,
                                                            const G2AStore* S, uint4* T4, uint8_t* tinf, G2JStore* QS) {
  DG_HI();
  const uint32_t gl = blockIdx.x * blockDim.x + threadIdx.x;
  __shared__ G2JStore s_acc[64];
  const uint32_t c = cnt[0], nq = (c + 3) / 4;
  if (gl == 0) cnt[1] = (nq + qpg - 1) / qpg;
  const uint32_t q = gl >> 1, side = gl & 1;
  if (q >= nq || q >= nqmax) return;
  const uint64_t seed = *seedp;
  uint32_t idx[4];
  uint64_t rho[4];
#pragma unroll
  for (uint32_t m = 0; m < 4; ++m) {
    const uint32_t j = 4 * q + m;
    idx[m] = j < c ? cand[j] : ~0u;
    rho[m] = j < c ? xr_rho(seed, idx[m]) : 0;
  }
  const size_t stride = 2 * (size_t)nqmax;
  auto member = [&](uint32_t m) {
    const uint32_t i = m == 0 ? idx[0] : m == 1 ? idx[1] : m == 2 ? idx[2] : idx[3];
    if (i == ~0u) return G2A{fp2_zero(), fp2_zero(), true};
    return side ? load_g2a(S[i]) : xr_q_aff(Q[i]);
  };
  auto getT = [&](uint32_t u) {
    G2A t;
    t.inf = tinf[u * stride + gl] != 0;
    rc_ld(T4 + u * RC_Q * stride + gl, stride, t.x, t.y);
    return t;
  };
  auto putT = [&](uint32_t u, const G2A& t) {
    tinf[u * stride + gl] = t.inf ? 1 : 0;
    rc_st(T4 + u * RC_Q * stride + gl, stride, t.inf ? fp2_zero() : t.x, t.inf ? fp2_zero() : t.y);
  };
  xq_sum4(member, rho, getT, putT, s_acc[threadIdx.x]);
  QS[gl] = s_acc[threadIdx.x];
}
#else
DG_KERNEL void __launch_bounds__(64, DG_CK_WAVES2) k_xq_sum(uint32_t nqmax, uint32_t qpg, const uint64_t* seedp,
                                                            uint32_t* cnt, const uint32_t* cand, const G2JStore* Q,
                                                            const G2AStore* S, uint4* T4, uint8_t* tinf, G2JStore* QS);
#endif
#if DG_TU_LIB
// the decoded items of [i0, i0 + n) of a failed batch (flag[0] == 0), compacted into cand (one atomic per wave, input
// order within a wave); none after a passed batch
DG_KERNEL void __launch_bounds__(256) k_xg_cand(uint32_t i0, uint32_t n, const uint32_t* flag, const uint8_t* status,
                                                uint32_t* cand, uint32_t* cnt) {
  DG_HI();
  const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  const bool on = g < n && !flag[0] && status[i0 + g] == DG_ST_OK_;
  const uint64_t m = __ballot(on);
  if (!m) return;
  const uint32_t lane = threadIdx.x & 63, first = (uint32_t)__ffsll((unsigned long long)m) - 1;
  uint32_t base = 0;
  if (lane == first) base = atomicAdd(&cnt[0], (uint32_t)__popcll(m));
  base = __shfl(base, (int)first);
  if (on) cand[base + (uint32_t)__popcll(m & ((1ull << lane) - 1))] = i0 + g;
}
// the verdicts of level `level` (good[g]: k_ck_final; gcnt: the launch's device count): a passed group leaves its rounds
// valid (their status is OK already), a failed group lists its rounds for level 3; a single check writes kyber's
// verdict.  xrc[level - 1] counts the checks (dg_isolation_counts).
DG_KERNEL void __launch_bounds__(128) k_xg_verdict(uint32_t level, uint32_t G, const uint32_t* gcnt, uint32_t qpg,
                                                   uint32_t* cnt, const uint8_t* good, const uint32_t* cand,
                                                   uint32_t* l3list, uint8_t* status, unsigned long long* xrc) {
  DG_HI();
  const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  if (ck_dead(g, G, gcnt)) return;
  atomicAdd(&xrc[level - 1], 1ull);
  const bool ok = good[g] != 0;
  if (level == 3) {
    status[l3list[g]] = ok ? DG_ST_OK_ : DG_ST_BAD_SIG_;
    return;
  }
  if (ok) return;
  const uint32_t c = cnt[0], j0 = 4 * g * qpg, j1 = j0 + 4 * qpg < c ? j0 + 4 * qpg : c;
  const uint32_t pos = atomicAdd(&cnt[3], j1 - j0);
  for (uint32_t j = j0; j < j1; ++j) l3list[pos + j - j0] = cand[j];
}
#endif
#endif

}  // namespace dg
