// HIP kernels of the threshold-BLS verify/aggregate path.  One item (round / partial) per lane; every
// kernel is compute-bound on 32-bit integer multiply-adds, HBM traffic is a few
// hundred bytes per item.
#pragma once
#include "h2c.h"
#include "pairing.h"
#include "fr.h"
#include "coop.h"

#ifndef DG_HOT_WAVES
#define DG_HOT_WAVES 2  // min waves per SIMD for the hot kernels: 256 VGPRs each (measured: 2 beats 1 by 6%)
#endif
#ifndef DG_TERMS_WAVES
#define DG_TERMS_WAVES DG_HOT_WAVES  // min waves per SIMD of Recover's MSM lanes (k_rc_straus, k_rs_sac)
#endif
#ifndef DG_BULK_WAVES
#define DG_BULK_WAVES 1  // min waves per SIMD for the other per-lane group-arithmetic kernels
#endif
#ifndef DG_COOP_WAVES
#define DG_COOP_WAVES 1  // min waves per SIMD for the cooperative (latency-bound) kernels
#endif
#ifndef DG_TU_HOT
#define DG_TU_HOT 0  // 1 in kernels_hot.hip: only the hot kernels are defined there (DESIGN.md §code generation)
#endif
#ifndef DG_TU_CHECK
#define DG_TU_CHECK 0  // 1 in kernels_check.hip: only the pairing-check pipeline of checks.h is defined there
#endif
#define DG_TU_LIB (!DG_TU_HOT && !DG_TU_CHECK)  // the library translation unit (drand_gpu.hip)

namespace dg {

// per-item status codes (mirror include/drand_gpu.h DG_ST_*)
constexpr uint8_t DG_ST_OK_ = 0, DG_ST_BAD_SIG_ = 1, DG_ST_SIG_DECODE_ = 2, DG_ST_BAD_INDEX_ = 3, DG_ST_PK_DECODE_ = 4,
                  DG_ST_NOT_ENOUGH_ = 5, DG_ST_NOT_EXAMINED_ = 255;

// ------------------------------------------------------------------------------------------ layouts
// Points in HBM: plain structs of Montgomery limbs (array-of-structs; the kernels are ALU-bound).
struct G2JStore {
  Fp2 x, y, z;
};
struct G2AStore {
  Fp2 x, y;
  uint32_t inf;
  uint32_t pad[3];
};
struct G1AStore {
  Fp x, y;
  uint32_t inf;
  uint32_t pad[3];
};

DGI G2J load_g2j(const G2JStore& s) { return G2J{s.x, s.y, s.z}; }
DGI void store_g2j(G2JStore& s, const G2J& p) {
  s.x = p.x;
  s.y = p.y;
  s.z = p.z;
}
DGI G2A load_g2a(const G2AStore& s) { return G2A{s.x, s.y, s.inf != 0}; }
DGI void store_g2a(G2AStore& s, const G2A& a) {
  s.x = a.x;
  s.y = a.y;
  s.inf = a.inf ? 1u : 0u;
}
DGI G1A load_g1a(const G1AStore& s) { return G1A{s.x, s.y, s.inf != 0}; }
DGI void store_g1a(G1AStore& s, const G1A& a) {
  s.x = a.x;
  s.y = a.y;
  s.inf = a.inf ? 1u : 0u;
}

// SHA-256(BE64 seed || BE64 i)
DGI void rlc_digest(uint64_t seed, uint64_t i, uint8_t d[32]) {
  Sha256 s;
  sha256_init(s);
  for (int b = 7; b >= 0; --b) sha256_byte(s, (uint8_t)(seed >> (8 * b)));
  for (int b = 7; b >= 0; --b) sha256_byte(s, (uint8_t)(i >> (8 * b)));
  sha256_final(s, d);
}

// 64-bit RLC coefficient for item i: first 8 bytes of SHA-256(seed || i), forced odd and non-zero
DGI uint64_t rlc_coeff(uint64_t seed, uint64_t i) {
  uint8_t d[32];
  rlc_digest(seed, i, d);
  uint64_t r = 0;
  for (int b = 0; b < 8; ++b) r = (r << 8) | d[b];
  return r | 1ull;
}

#if defined(__HIP__)
#define DG_KERNEL extern "C" __global__
// Latency-bound kernels (a few waves on a chip shared with other batches: the cooperative tail, the check pipeline of
// the isolation passes) raise their waves' issue priority, so the throughput waves on the same SIMDs fill the gaps
// instead of stretching the latency-bound chain (DG_PRIO=0: equal priority, A/B)
#ifndef DG_PRIO
#define DG_PRIO 1
#endif
#if DG_PRIO && defined(__HIP_DEVICE_COMPILE__)
#define DG_HI() __builtin_amdgcn_s_setprio(3)
#else
#define DG_HI() ((void)0)
#endif

// A1: beacon messages
#if DG_TU_LIB
DG_KERNEL void __launch_bounds__(256) k_beacon_msgs(uint32_t n, const uint64_t* prev_round, const uint64_t* round,
                                                    const uint8_t* prev_sigs, const uint32_t* off, uint8_t* out32) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t a = off[i], b = off[i + 1];
  beacon_message(out32 + 32ull * i, prev_sigs + a, b - a, prev_round[i], round[i]);
}
#endif

// A2: randomness
#if DG_TU_LIB
DG_KERNEL void __launch_bounds__(256) k_randomness(uint32_t n, const uint8_t* sigs96, uint8_t* out32) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  Sha256 s;
  sha256_init(s);
  sha256_update(s, sigs96 + 96ull * i, 96);
  sha256_final(s, out32 + 32ull * i);
}
#endif

// A13: link check
#if DG_TU_LIB
DG_KERNEL void __launch_bounds__(256) k_links(uint32_t n, uint64_t cur_round, const uint8_t* cur_sig, uint32_t cur_len,
                                              const uint64_t* prev_round, const uint64_t* round,
                                              const uint8_t* prev_sigs, const uint32_t* off, const uint8_t* sigs96,
                                              uint8_t* out) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint64_t cr = i == 0 ? cur_round : round[i - 1];
  const uint8_t* cs = i == 0 ? cur_sig : sigs96 + 96ull * (i - 1);
  uint32_t cl = i == 0 ? cur_len : 96;
  uint32_t a = off[i], b = off[i + 1];
  bool ok = round[i] > cr && prev_round[i] == cr && (b - a) == cl;
  if (ok)
    for (uint32_t k = 0; k < cl; ++k) ok = ok && prev_sigs[a + k] == cs[k];
  out[i] = ok ? 0 : 1;
}
#endif

// A9: full hash-to-G2, compressed
#if DG_TU_LIB
DG_KERNEL void __launch_bounds__(128) k_hash_to_g2(uint32_t n, const uint8_t* msgs, uint32_t msg_len,
                                                   const uint8_t* dst, uint32_t dst_len, uint8_t* out96) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  G2J h = hash_to_g2(msgs + (size_t)msg_len * i, msg_len, dst, dst_len);
  g2_compress_aff(out96 + 96ull * i, g2_to_aff(h));
}
#endif



// G1 decode (keys, commits), with subgroup check
#if DG_TU_LIB
DG_KERNEL void __launch_bounds__(64) k_decode_g1(uint32_t n, const uint8_t* in48, G1AStore* out, uint8_t* status) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  G1A a;
  bool ok = g1_decompress(a, in48 + 48ull * i, true);
  if (!ok) a = G1A{fp_zero(), fp_zero(), true};
  store_g1a(out[i], a);
  status[i] = ok ? DG_ST_OK_ : DG_ST_PK_DECODE_;
}
#endif

// ------------------------------------------------------------------ batch verification engine
// Items are (round r, key slot s) pairs laid out round-major, k items per round (k = 1 for chain
// verification, k = partials per round for VerifyPartial / Recover).  Soundness of the batch:
// the random linear combination uses coefficient alpha_r * beta_s for item (r, s), so the batch
// equation is  prod_s e(beta_s X_s, h_eff(sum_{r in R_s} alpha_r Q_r)) * e(-g1, sum_r alpha_r sum_s beta_s S_rs) = 1,
// a bilinear form alpha^T E beta in the per-item errors E_rs (Schwartz-Zippel bound 2 / 2^64).  An item
// whose (r, s) cell is already taken (a second partial with the same index in one round) is checked
// on its own instead.  With a single key slot beta = 1.
DGI uint64_t rlc_alpha(uint64_t seed, uint64_t r) { return rlc_coeff(seed, r); }
DGI uint64_t rlc_beta(uint64_t seed, uint64_t s) { return rlc_coeff(~seed, s); }

// [k]P for a small scalar (< 2^nbits), MSB first
template <class F>
DGN Jac<F> jac_mul_small(const Jac<F>& p, uint32_t k) {
  Jac<F> acc = jac_infinity<F>();
  int top = 31;
  while (top >= 0 && !((k >> top) & 1)) --top;
  for (int b = top; b >= 0; --b) {
    acc = jac_dbl(acc);
    if ((k >> b) & 1) acc = jac_add(acc, p);
  }
  return acc;
}

DGI uint32_t be16(const uint8_t* p) { return (uint32_t)p[0] << 8 | p[1]; }

// A12: PubPoly.Eval(idx) = sum_j C_j x^j at x = idx + 1 (Horner), affine (+ compressed when out48)
#if DG_TU_LIB
DG_KERNEL void __launch_bounds__(64) k_pubpoly_eval(uint32_t n, uint32_t t, const G1AStore* commits,
                                                    const uint8_t* commit_status, const uint32_t* idx,
                                                    G1AStore* out, uint8_t* out_status, uint8_t* out48) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  bool ok = true;
  for (uint32_t j = 0; j < t; ++j) ok = ok && commit_status[j] == DG_ST_OK_;
  G1A a{fp_zero(), fp_zero(), true};
  if (ok) {
    uint32_t x = idx[i] + 1;
    G1J acc = jac_from_aff(load_g1a(commits[t - 1]));
    for (int j = (int)t - 2; j >= 0; --j) acc = jac_add(jac_mul_small(acc, x), jac_from_aff(load_g1a(commits[j])));
    a = g1_to_aff(acc);
  }
  store_g1a(out[i], a);
  if (out_status) out_status[i] = ok ? DG_ST_OK_ : DG_ST_PK_DECODE_;
  if (out48) g1_compress_aff(out48 + 48ull * i, a);
}
#endif


// U_i = beta_slot S_i for batch items, O otherwise
#if DG_TU_LIB
DG_KERNEL void __launch_bounds__(128, DG_BULK_WAVES) k_scale_items(uint32_t n, uint32_t nslots, const uint64_t* seedp,
                                                    const uint32_t* item_slot, const G2AStore* S,
                                                    const uint8_t* status, const uint8_t* isolate, G2JStore* U) {
  const uint64_t seed = *seedp;
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  G2J u = jac_infinity<Fp2>();
  if (status[i] == DG_ST_OK_ && !isolate[i]) {
    u = jac_from_aff(load_g2a(S[i]));
    if (nslots > 1) u = jac_mul_u64(u, rlc_beta(seed, item_slot ? item_slot[i] : 0u));
  }
  store_g2j(U[i], u);
}
#endif

// per round r: V_r = sum_j U_{r,j} over its batch items, active[r] = (any batch item); with several
// key slots also A_r = alpha_r Q_r, but only for an active round with an empty (r, s) cell: the hash side
// of key s is K_s = K - C_s with K = sum over the active rounds of alpha_r Q_r (one Pippenger MSM, msm.h)
// and C_s = sum of A_r over the active rounds without an item of s (k_key_accum) -- nothing when every
// share is present in every round
// (hot TU: the running sums in LDS, additions and the 64-bit scalar multiplication inlined with serialised products,
// curve.h g2_add_lds / g2_dbl_lds -- round 3 ran it in the library TU with out-of-line products)
#if DG_TU_HOT
DG_KERNEL void __launch_bounds__(128, DG_HOT_WAVES) k_round_combine(uint32_t R, uint32_t k, uint32_t nslots, const uint64_t* seedp,
                                                      const G2JStore* U, const uint8_t* status,
                                                      const uint8_t* isolate, const G2JStore* Q, const uint32_t* cell,
                                                      G2JStore* V, G2JStore* A, uint8_t* active) {
  const uint64_t seed = *seedp;
  __shared__ G2JStore s_acc[128];
  uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= R) return;
  G2JStore& v = s_acc[threadIdx.x];
  v.x = fp2_zero();
  v.y = fp2_zero();
  v.z = fp2_zero();
  bool any = false;
  for (uint32_t j = 0; j < k; ++j) {
    size_t i = (size_t)r * k + j;
    if (status[i] == DG_ST_OK_ && !isolate[i]) {
      if (U) g2_add_lds(v, load_g2j(U[i]));
      any = true;
    }
  }
  if (V) V[r] = v;  // V (and U) only on the single-key path; the keyed MSM reads S directly
  active[r] = any ? 1 : 0;
  if (nslots > 1) {
    bool gap = false;
    for (uint32_t s = 0; any && s < nslots && !gap; ++s) gap = cell[(size_t)r * nslots + s] == 0u;
    if (gap) {  // A_r = alpha_r Q_r, MSB first
      const uint64_t a = rlc_alpha(seed, r);
      const G2J q = load_g2j(Q[r]);
      v.x = fp2_zero();
      v.y = fp2_zero();
      v.z = fp2_zero();
#pragma unroll 1
      for (int b = 63; b >= 0; --b) {
        g2_dbl_lds(v);
        if ((a >> b) & 1) g2_add_lds(v, q);
      }
      A[r] = v;
    }
  }
}
#elif defined(__HIP__)
DG_KERNEL void __launch_bounds__(128, DG_HOT_WAVES) k_round_combine(uint32_t R, uint32_t k, uint32_t nslots, const uint64_t* seedp,
                                                      const G2JStore* U, const uint8_t* status,
                                                      const uint8_t* isolate, const G2JStore* Q, const uint32_t* cell,
                                                      G2JStore* V, G2JStore* A, uint8_t* active);
#endif

// Kp[s * nchunks + c] = -(sum of A_r over the active rounds r in chunk c without an item of key s), so the
// row sums are -C_s (k_round_combine)
#if DG_TU_HOT
DG_KERNEL void __launch_bounds__(128, DG_HOT_WAVES) k_key_accum(uint32_t R, uint32_t nslots, uint32_t chunk, uint32_t nchunks,
                                                  const uint32_t* cell, const uint8_t* active, const G2JStore* A,
                                                  G2JStore* Kp) {
  __shared__ G2JStore s_acc[128];
  uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= nslots * nchunks) return;
  uint32_t s = g / nchunks, c = g % nchunks;
  uint32_t a = c * chunk, b = a + chunk < R ? a + chunk : R;
  G2JStore& acc = s_acc[threadIdx.x];
  acc.x = fp2_zero();
  acc.y = fp2_zero();
  acc.z = fp2_zero();
  for (uint32_t r = a; r < b; ++r)
    if (active[r] && !cell[(size_t)r * nslots + s]) g2_add_lds(acc, load_g2j(A[r]));
  store_g2j(Kp[g], jac_neg(load_g2j(acc)));
}
// Xc = sum_s beta_s X_s over the key slots with a decoded key: per-lane 64-bit products, LDS tree sum.  One workgroup
// whose ~2 ms are latency (64 dependent doublings per lane, one wave per SIMD; inline products did not change it):
// batch_verify runs it on a side stream beside the keyed MSM, off the batch's critical path.
DG_KERNEL void __launch_bounds__(256) k_key_combine(uint32_t nslots, const uint64_t* seedp, const G1AStore* keys,
                                                   const uint8_t* key_status, G1AStore* out) {
  const uint64_t seed = *seedp;
  __shared__ G1J part[256];
  const uint32_t t = threadIdx.x;
  G1J acc = jac_infinity<Fp>();
  for (uint32_t s = t; s < nslots; s += 256) {
    G1A a = load_g1a(keys[s]);
    if (key_status[s] != DG_ST_OK_ || a.inf) continue;
    acc = jac_add(acc, jac_mul_u64(jac_from_aff(a), rlc_beta(seed, s)));
  }
  part[t] = acc;
  __syncthreads();
  for (uint32_t w = 128; w > 0; w >>= 1) {
    if (t < w) part[t] = jac_add(part[t], part[t + w]);
    __syncthreads();
  }
  if (t == 0) store_g1a(out[0], g1_to_aff(part[0]));
}
#elif defined(__HIP__)
DG_KERNEL void __launch_bounds__(128, DG_HOT_WAVES) k_key_accum(uint32_t R, uint32_t nslots, uint32_t chunk, uint32_t nchunks,
                                                  const uint32_t* cell, const uint8_t* active, const G2JStore* A,
                                                  G2JStore* Kp);
DG_KERNEL void __launch_bounds__(256) k_key_combine(uint32_t nslots, const uint64_t* seedp, const G1AStore* keys,
                                                   const uint8_t* key_status, G1AStore* out);
#endif


// Pair s on one 128-lane workgroup (coop.h): P side and Q side prepared cooperatively (for key pairs the
// hash-side sum is cofactor-cleared here, once per key and batch), then the cooperative Miller loop.
// Pairs: (beta_s X_s, h_eff K_s) for s < nslots, (-g1, T) for s == nslots; with several keys (Kc given)
// K_s = -C_s and one more pair (Xc, h_eff Kc), Xc = sum_s beta_s X_s: prod_s e(beta_s X_s, h(Kc - C_s)).
// f[s] = 1 when a side is the identity (every correction pair when all shares are present).
#if DG_TU_LIB
// Workgroups npairs.. (when win != null) run the batched subgroup check of window sum win[blockIdx.x - npairs]
// instead (co_subgroup_check, *sub_fail = 1 on failure): independent of the pairs, so they share the launch.
DG_KERNEL void __launch_bounds__(128, DG_COOP_WAVES) k_pair_miller_coop(uint32_t nslots, const uint64_t* seedp, const G1AStore* keys,
                                                         const G2JStore* K, const G2JStore* T, const G1AStore* Xc,
                                                         const G2JStore* Kc, Fp12* f, uint32_t npairs,
                                                         const G2JStore* win, uint32_t* sub_fail) {
  DG_HI();
  const uint64_t seed = *seedp;
  __shared__ CoGT gt;
  __shared__ CoML ml;
  __shared__ CoG2Tmp g2t;
  __shared__ CoG2 Kp, tp[4];
  __shared__ Fp12W F, L;
  __shared__ uint32_t skip;
  const uint32_t s = blockIdx.x;
  if (s >= npairs) {
    co_subgroup_check(win + (s - npairs), &Kp, &tp[0], &tp[1], &g2t, sub_fail);
    return;
  }
  if (s < nslots || s == nslots + 1) {
    CO_SERIAL({
      G2J k = load_g2j(s < nslots ? K[s] : Kc[0]);
      Kp = CoG2{k.x, k.y, k.z};
      skip = jac_is_inf(k) ? 1u : 0u;
      if (!skip) {
        G1A pa = load_g1a(s < nslots ? keys[s] : Xc[0]);  // decoded keys are affine already; one key: beta = 1
        if (s < nslots && nslots > 1) pa = g1_to_aff(jac_mul_u64(jac_from_aff(pa), rlc_beta(seed, s)));
        ml.px = pa.x;
        ml.py = pa.y;
        skip = pa.inf ? 1u : 0u;
      }
    });
    if (skip) {
      if (threadIdx.x == 0) f[s] = fp12_one();
      return;
    }
    co_g2_clear_cofactor(&Kp, tp, &g2t);
    CO_SERIAL({
      G2A qa = g2_to_aff(G2J{Kp.x, Kp.y, Kp.z});
      ml.qx = qa.x;
      ml.qy = qa.y;
      skip |= qa.inf ? 1u : 0u;
    });
  } else {
    CO_SERIAL({
      ml.px = fp_const(G1_GEN_X);
      ml.py = fp_const(G1_GEN_NEG_Y);
      G2A qa = g2_to_aff(load_g2j(T[0]));
      ml.qx = qa.x;
      ml.qy = qa.y;
      skip = qa.inf ? 1u : 0u;
    });
  }
  if (skip) {
    if (threadIdx.x == 0) f[s] = fp12_one();
    return;
  }
  co_miller_loop(&F, &L, &ml, &gt);
  if (threadIdx.x < 6) ((Fp2*)&f[s])[(threadIdx.x & 1) * 3 + threadIdx.x / 2] = F.e[threadIdx.x];
}
#endif

// product of the npairs Miller values and one final exponentiation on one 128-lane workgroup
#if DG_TU_LIB
// ok = (product of the Miller values, final-exponentiated, is 1) and no subgroup failure (*sub_fail == 0)
DG_KERNEL void __launch_bounds__(128, DG_COOP_WAVES) k_final_coop(uint32_t npairs, const Fp12* f, uint32_t* ok,
                                                                  const uint32_t* sub_fail) {
  DG_HI();
  __shared__ CoGT gt;
  __shared__ Fp12W F, G, S[7];
  const int t = threadIdx.x;
  co_gt_init(&gt);
  if (t < 6) F.e[t] = ((const Fp2*)&f[0])[(t & 1) * 3 + t / 2];
  __syncthreads();
  for (uint32_t s = 1; s < npairs; ++s) {
    if (t < 6) G.e[t] = ((const Fp2*)&f[s])[(t & 1) * 3 + t / 2];
    __syncthreads();
    co_fp12_mul(&F, &F, &G, &gt);
  }
  co_final_exp_cubed(&F, S, &gt);
  if (t == 0) {
    bool one = fp2_eq(F.e[0], fp2_one());
    for (int k = 1; k < 6; ++k) one = one && fp2_is_zero(F.e[k]);
    *ok = one && *sub_fail == 0u ? 1u : 0u;
  }
}
#endif

// ---- Group tests over the examined prefix (checks.h).  With a corrupted fraction f of the shares, one pairing check
// per examined item is more than Recover needs: up to GRP consecutive unverified items of one round are
// checked together, e(sum_i rho_i X_i, H_r) == e(g1, sum_i rho_i S_i) with independent 64-bit rho_i from the
// batch's bound seed.  Every S_i is in G2 (subgroup-checked by k_ck_sub) and H_r is in G2, so a
// member with x_i H_r != S_i makes the sum vanish for at most one rho_i value mod r: a group with a bad
// member passes with probability <= 2^-63 (rho_i is odd: 2^63 values).  A passed group gives every member kyber's nil verdict; the
// members of a failed group are marked for their own check (fin = FIN_RECHECK) in the next pass, which
// decides every verdict Recover reads.  At f = 10% and GRP = 4 that is ~0.6 pairing checks per item.
constexpr uint32_t GRP = 4;
constexpr uint8_t FIN_PENDING = 0, FIN_DONE = 1, FIN_RECHECK = 2;
constexpr uint64_t GROUP_TAG = 0x67726f7570746573ull;  // domain of rho_i, apart from alpha_r and beta_s
#if DG_TU_CHECK || !defined(__HIP__)
// the single-lane reference of the pipeline's checks (host builds: tests/native/hostcheck.cpp)
DGN Fp12 miller_loop2(const G1A* P, const G2A* Q, int np) { return miller_loop<2>(P, Q, np); }
// e(x, h) * e(-g1, s) == 1 (the identity's pairings dropped): kyber's bls.Verify equation
DGN bool pair_check(const G1A& x, const G2A& h, const G2A& s) {
  G1A P[2];
  G2A Qa[2];
  int np = 0;
  if (!x.inf && !h.inf) {
    P[np] = x;
    Qa[np] = h;
    ++np;
  }
  if (!s.inf) {
    P[np] = G1A{fp_const(G1_GEN_X), fp_const(G1_GEN_NEG_Y), false};
    Qa[np] = s;
    ++np;
  }
  return np == 0 ? true : fp12_is_one(final_exp_cubed(miller_loop2(P, Qa, np)));
}
// the members' G1 weighted sum a = sum rho_i X_i (the G2 sum b = sum rho_i S_i is left to checks.h's table kernels,
// k_ck_tab_*, k_ck_sac, except for a single share: b = its sigma); members failing the subgroup check are decided here
// (decode error) and left out.  Returns the live members (their item indices in live[], coefficients in rho_out[]).
DGN uint32_t group_combine(const uint32_t* mem, uint32_t n, uint64_t seed, const G1AStore* keys,
                             const uint32_t* item_slot, const G2AStore* S, uint8_t* status, uint8_t* fin,
                             uint32_t subgroup, G1A& a, G2A& b, uint32_t* live, uint64_t* rho_out) {
  G1J xp[GRP];
  uint64_t rho[GRP];
  uint32_t nl = 0;
  for (uint32_t m = 0; m < n; ++m) {
    const uint32_t i = mem[m];
    if (fin[i] == FIN_DONE) continue;  // decided before the check (checks.h k_ck_sub: outside G2)
    const G2A s = load_g2a(S[i]);
    // (a recheck was subgroup-checked by its group)
    if (subgroup && fin[i] != FIN_RECHECK && !s.inf && !g2_in_subgroup_aff(s.x, s.y)) {
      status[i] = DG_ST_SIG_DECODE_;
      fin[i] = FIN_DONE;
      continue;
    }
    if (n == 1) {  // a share's own check: its key and signature as they are
      a = load_g1a(keys[item_slot ? item_slot[i] : 0u]);
      b = s;
      live[0] = i;
      return 1;
    }
    xp[nl] = jac_from_aff(load_g1a(keys[item_slot ? item_slot[i] : 0u]));
    rho[nl] = rlc_coeff(seed ^ GROUP_TAG, i);
    live[nl++] = i;
  }
  for (uint32_t m = nl; m < GRP; ++m) {
    xp[m] = jac_infinity<Fp>();
    rho[m] = 0;
  }
  if (rho_out)
    for (uint32_t m = 0; m < GRP; ++m) rho_out[m] = rho[m];
  if (nl) a = g1_to_aff(jac_msm4_sac(xp, rho));
  (void)b;
  return nl;
}
#endif
#if DG_TU_LIB
// ---- Recover's window (drand_gpu.hip recover_windowed).  kyber's tbls.Recover verifies the partials of a
// round in input order and stops at the t-th valid one (beacon/beacon.go:488), so the batch equation first
// covers only the first w = t partials of every round; the rest are decoded and checked only for the rounds
// whose window did not yield t valid shares.  Rows of a round-major table move between the R x k layout of
// the input and the R x w layout of a window: dst[(r kout + jout + j) ne + e] = src[(r kin + jin + j) ne + e].
template <typename T>
__global__ void __launch_bounds__(256) k_rows(uint32_t R, uint32_t w, uint32_t ne, uint32_t kin, uint32_t jin,
                                            uint32_t kout, uint32_t jout, const T* src, T* dst) {
  const size_t n = (size_t)R * w * ne;
  const size_t x = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (x >= n) return;
  const size_t item = x / ne;
  const uint32_t e = (uint32_t)(x - item * ne), r = (uint32_t)(item / w), j = (uint32_t)(item - (size_t)r * w);
  dst[((size_t)r * kout + jout + j) * ne + e] = src[((size_t)r * kin + jin + j) * ne + e];
}
// statuses of window items (r, j0 + j), j < w, into the R x k table, and whether each verdict is final: a decode
// failure, or (window batch: flag != null) a passed batch equation and not isolated.  inc |= 1: an item is
// pending (it needs its own check); inc |= 2: a window item is not valid while shares lie beyond the window
// (kyber would go on to the next partial).
DG_KERNEL void __launch_bounds__(256) k_window_fin(uint32_t R, uint32_t k, uint32_t j0, uint32_t w, const uint32_t* flag,
                                                  const uint8_t* iso, const uint8_t* st_w, uint8_t* status,
                                                  uint8_t* fin, uint32_t* inc) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= R * w) return;
  const uint32_t r = i / w, f = r * k + j0 + (i - r * w);
  const uint8_t st = st_w[i];
  const bool done = st != DG_ST_OK_ || (flag && flag[0] && !iso[i]);
  status[f] = st;
  fin[f] = done ? FIN_DONE : FIN_PENDING;
  uint32_t m = done ? 0u : 1u;
  if (flag && st != DG_ST_OK_ && w < k) m |= 2u;
  if (m) atomicOr(inc, m);
}
// per round: scanning in input order, the unverified items up to the point where the round would reach
// t + margin valid shares if every fresh unverified item were valid and every member of a failed group (bad
// with probability ~1/3 at 10% corruption) counted one half -- a speculative margin, so that few rounds
// need another pass (each costs one pairing's latency, ~60 ms); checking shares beyond the t-th valid one is
// harmless, k_recover_select reports them not examined.  `all` (the last pass): every unverified item before
// the t-th verified valid one, which makes the statuses Recover reads exact.  Into groups: glist[0] = count,
// group g = glist[4 + 4g .. 8 + 4g) (item indices, ~0u = empty).  Consecutive fresh items of a round share a
// group of up to `grp`; members of a failed group, and every item in the last pass, go alone.
DG_KERNEL void __launch_bounds__(128) k_prefix_groups(uint32_t R, uint32_t k, uint32_t t, uint32_t all, uint32_t grp,
                                                     uint32_t margin, const uint8_t* status, const uint8_t* fin,
                                                     uint32_t* glist) {
  uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= R) return;
  uint32_t valid = 0, fresh = 0, rech = 0, cur[GRP], nc = 0;
  auto emit = [&](const uint32_t* m, uint32_t c) {
    uint32_t* g = glist + 4 + 4 * (size_t)atomicAdd(&glist[0], 1u);
    for (uint32_t q = 0; q < GRP; ++q) g[q] = q < c ? m[q] : ~0u;
  };
  for (uint32_t j = 0; j < k; ++j) {
    size_t i = (size_t)r * k + j;
    if (valid >= t || (!all && 2 * (valid + fresh) + rech >= 2 * (t + margin))) break;
    if (fin[i] == FIN_DONE) {
      if (status[i] == DG_ST_OK_) ++valid;
      continue;
    }
    if (fin[i] == FIN_RECHECK)
      ++rech;
    else
      ++fresh;
    const uint32_t one = (uint32_t)i;
    if (all || grp < 2 || fin[i] == FIN_RECHECK) {
      emit(&one, 1);
    } else {
      cur[nc++] = (uint32_t)i;
      if (nc == grp) {
        emit(cur, nc);
        nc = 0;
      }
    }
  }
  if (nc) emit(cur, nc);
}
#endif

// Key-slot statistics of a VerifyPartial / Recover batch (drand_gpu.hip verify_partials_dev): per share
// index its number of partials and its first position; then each item's slot from the host's slot table.
#if DG_TU_LIB
// (count: only the items of each round's first w of k, the window of a Recover batch; first: every item)
DG_KERNEL void __launch_bounds__(256) k_index_scan(uint32_t n, uint32_t k, uint32_t w, const uint8_t* partials98,
                                                  uint32_t* count, uint32_t* first) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t idx = (uint32_t)partials98[98ull * i] << 8 | partials98[98ull * i + 1];
  if (i % k < w) atomicAdd(&count[idx], 1u);
  if (i < first[idx]) atomicMin(&first[idx], i);
}
DG_KERNEL void __launch_bounds__(256) k_item_slots(uint32_t n, const uint8_t* partials98, const int32_t* slot_of,
                                                  uint32_t* item_slot) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  item_slot[i] = (uint32_t)slot_of[(uint32_t)partials98[98ull * i] << 8 | partials98[98ull * i + 1]];
}
#endif

// *flag |= 1 if any byte of v[0..n) is non-zero
#if DG_TU_LIB
DG_KERNEL void __launch_bounds__(256) k_any(uint32_t n, const uint8_t* v, uint32_t* flag) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n && v[i]) atomicOr(flag, 1u);
}
// batches whose random-linear-combination check failed or that isolated items (the per-item pass ran):
// stream-ordered diagnostics counter, read with dg_fallback_count
DG_KERNEL void __launch_bounds__(64) k_count_fallback(const uint32_t* flag, unsigned long long* counter) {
  if (threadIdx.x == 0 && (!flag[0] || flag[1])) atomicAdd(counter, 1ull);
}

struct Seed0 {
  uint32_t w[8];
};
// ---- Binding the batch coefficients to the batch (Fiat-Shamir).  alpha_r, beta_s and the test-window
// digits of the batched subgroup check are keyed by seed' = SHA-256(seed0 || D)[0..8), where seed0 =
// SHA-256(BE64 seed || key bytes) (host) and D is a SHA-256 tree over every item (message and signature
// record).  A caller-known seed therefore does not let anyone choose items whose errors cancel in the
// batch equation: changing any item changes every coefficient.
// d_i = SHA-256(BE32 i || msg_{i / k} || record_i), record_i = the `stride` bytes at recs + stride * i
DG_KERNEL void __launch_bounds__(128) k_digest_items(uint32_t n, uint32_t k, const uint8_t* msgs, uint32_t msg_len,
                                                     const uint8_t* recs, uint32_t stride, uint8_t* out32) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  Sha256 s;
  sha256_init(s);
  for (int b = 3; b >= 0; --b) sha256_byte(s, (uint8_t)(i >> (8 * b)));
  sha256_update(s, msgs + (size_t)msg_len * (i / k), msg_len);
  sha256_update(s, recs + (size_t)stride * i, stride);
  sha256_final(s, out32 + 32ull * i);
}
// one tree level: out_j = SHA-256(in_{64 j} || ... || in_{min(64 j + 63, n - 1)}) (32 B digests, word-wise:
// two digests per block, then the padding)
DGI uint32_t ld_be32(const uint8_t* p) {
  return (uint32_t)p[0] << 24 | (uint32_t)p[1] << 16 | (uint32_t)p[2] << 8 | p[3];
}
DG_KERNEL void __launch_bounds__(128) k_digest_level(uint32_t n, const uint8_t* in32, uint8_t* out32) {
  uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t a = 64 * j;
  if (a >= n) return;
  uint32_t b = a + 64 < n ? a + 64 : n;
  uint32_t h[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a, 0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
  uint32_t w[16];
  uint32_t q = a;
  for (; q + 1 < b; q += 2) {
    const uint8_t* p = in32 + 32ull * q;
#pragma unroll
    for (int t = 0; t < 16; ++t) w[t] = ld_be32(p + 4 * t);
    sha256_compress(h, w);
  }
  const bool odd = q < b;
  const uint8_t* p = in32 + 32ull * q;
#pragma unroll
  for (int t = 0; t < 8; ++t) w[t] = odd ? ld_be32(p + 4 * t) : 0u;
  w[odd ? 8 : 0] = 0x80000000u;
#pragma unroll
  for (int t = 1; t < 15; ++t)
    if (t != 8) w[t] = (odd && t < 8) ? w[t] : 0u;
  if (!odd) w[8] = 0u;
  w[15] = 256u * (b - a);
  sha256_compress(h, w);
#pragma unroll
  for (int t = 0; t < 8; ++t) {
    uint8_t* o = out32 + 32ull * j + 4 * t;
    o[0] = (uint8_t)(h[t] >> 24);
    o[1] = (uint8_t)(h[t] >> 16);
    o[2] = (uint8_t)(h[t] >> 8);
    o[3] = (uint8_t)h[t];
  }
}
// *seed_out = the first 8 bytes of SHA-256(seed0 || D), forced non-zero (seed0 as 8 big-endian words, passed by
// value; one block of 64 bytes plus the padding block)
DG_KERNEL void __launch_bounds__(64) k_digest_seed(Seed0 s0, const uint8_t* d32, uint64_t* seed_out) {
  if (threadIdx.x != 0) return;
  uint32_t h[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a, 0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
  uint32_t w[16];
#pragma unroll
  for (int t = 0; t < 8; ++t) {
    w[t] = s0.w[t];
    w[8 + t] = ld_be32(d32 + 4 * t);
  }
  sha256_compress(h, w);
#pragma unroll
  for (int t = 0; t < 16; ++t) w[t] = 0;
  w[0] = 0x80000000u;
  w[15] = 512u;
  sha256_compress(h, w);
  const uint64_t v = (uint64_t)h[0] << 32 | h[1];
  *seed_out = v ? v : 1ull;
}
#endif

// ------------------------------------------------------------------ Recover (A6)
// per round: the first t items (input order) that passed VerifyPartial, sorted by index, duplicates
// collapsed (kyber xyCommit); round_status NOT_ENOUGH if fewer than t distinct remain.  share_status
// = the verify status of every item examined, NOT_EXAMINED after the t-th collected one.
#if DG_TU_LIB
DG_KERNEL void __launch_bounds__(128) k_recover_select(uint32_t R, uint32_t k, uint32_t t, const uint8_t* partials,
                                                       const uint8_t* status, uint32_t* sel, uint32_t* selidx,
                                                       uint8_t* round_status, uint8_t* share_status) {
  uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= R) return;
  uint32_t* ps = sel + (size_t)r * t;
  uint32_t* pi = selidx + (size_t)r * t;
  uint32_t got = 0;
  for (uint32_t j = 0; j < k; ++j) {
    size_t i = (size_t)r * k + j;
    if (got >= t) {
      share_status[i] = DG_ST_NOT_EXAMINED_;
      continue;
    }
    uint8_t st = status[i];
    share_status[i] = st;
    if (st != DG_ST_OK_) continue;
    uint32_t idx = be16(partials + 98 * i);
    // insertion by index (stable: the earlier of two equal indices stays first)
    uint32_t m = got;
    while (m > 0 && pi[m - 1] > idx) {
      pi[m] = pi[m - 1];
      ps[m] = ps[m - 1];
      --m;
    }
    pi[m] = idx;
    ps[m] = j;
    ++got;
  }
  uint32_t distinct = 0;
  for (uint32_t m = 0; m < got; ++m) {
    if (m > 0 && pi[m] == pi[m - 1]) continue;
    pi[distinct] = pi[m];
    ps[distinct] = ps[m];
    ++distinct;
  }
  round_status[r] = distinct >= t ? DG_ST_OK_ : DG_ST_NOT_ENOUGH_;
}
#endif

// Recover with known VerifyPartial verdicts (dg_recover_verified, the live round: beacon/beacon.go:148 has
// already verified every partial the round cache holds, :488 would re-verify them): every sigma is decoded by the
// phase kernels (drand_gpu.hip decode_items, no subgroup check: an OK verdict already implies it), then this carries
// the verdicts -- an item whose verdict is not OK takes that verdict and the identity; an OK one keeps its decode
// status (a sigma that no longer decodes is a decode error).  Round 3 decoded with one single-lane g2_decompress
// per item (87 ms for 6.4 M partials).
#if DG_TU_LIB
DG_KERNEL void __launch_bounds__(128) k_merge_verified(uint32_t n, const uint8_t* vst, G2AStore* S, uint8_t* status) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint8_t v = vst[i];
  if (v != DG_ST_OK_) {
    store_g2a(S[i], G2A{fp2_zero(), fp2_zero(), true});
    status[i] = v;
  }
}
#endif

// compress points (zeros where status != OK)
#if DG_TU_LIB
DG_KERNEL void __launch_bounds__(128) k_compress_g2(uint32_t n, const G2JStore* P, const uint8_t* st, uint8_t* out96) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  if (st && st[i] != DG_ST_OK_) {
    for (int b = 0; b < 96; ++b) out96[96ull * i + b] = 0;
    return;
  }
  g2_compress_aff(out96 + 96ull * i, g2_to_aff(load_g2j(P[i])));
}
#endif

// A7: bls.Sign / tbls.Sign -- x * H(m); scalars are 32 B big-endian (< r)
#if DG_TU_LIB
DG_KERNEL void __launch_bounds__(128) k_sign(uint32_t n, const uint8_t* sc32, const uint16_t* index, const uint8_t* msgs,
                                             uint32_t msg_len, const uint8_t* dst, uint32_t dst_len, uint8_t* out) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t kl[8];
  const uint8_t* s = sc32 + 32ull * i;
  for (int w = 0; w < 8; ++w) {
    const uint8_t* q = s + 28 - 4 * w;
    kl[w] = (uint32_t)q[0] << 24 | (uint32_t)q[1] << 16 | (uint32_t)q[2] << 8 | q[3];
  }
  G2J h = hash_to_g2(msgs + (size_t)msg_len * i, msg_len, dst, dst_len);
  G2A sig = g2_to_aff(g2_mul_u256_psi(g2_to_aff(h), kl));
  uint32_t rec = index ? 98u : 96u;
  uint8_t* o = out + (size_t)rec * i;
  if (index) {
    o[0] = (uint8_t)(index[i] >> 8);
    o[1] = (uint8_t)index[i];
    o += 2;
  }
  g2_compress_aff(o, sig);
}
#endif
#endif

}  // namespace dg

#include "phases.h"
#include "msm.h"
#include "recover.h"
#include "checks.h"
#include "xr.h"
