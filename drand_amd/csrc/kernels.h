// HIP kernels of the threshold-BLS verify/aggregate path.  One item (round / partial) per lane; every
// kernel is compute-bound on 32-bit integer multiply-adds, HBM traffic is a few
// hundred bytes per item.
#pragma once
#include "h2c.h"
#include "pairing.h"

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

// 64-bit RLC coefficient for item i: first 8 bytes of SHA-256(seed || i), forced odd and non-zero
DGI uint64_t rlc_coeff(uint64_t seed, uint64_t i) {
  Sha256 s;
  sha256_init(s);
  for (int b = 7; b >= 0; --b) sha256_byte(s, (uint8_t)(seed >> (8 * b)));
  for (int b = 7; b >= 0; --b) sha256_byte(s, (uint8_t)(i >> (8 * b)));
  uint8_t d[32];
  sha256_final(s, d);
  uint64_t r = 0;
  for (int b = 0; b < 8; ++b) r = (r << 8) | d[b];
  return r | 1ull;
}

#if defined(__HIP__)
#define DG_KERNEL extern "C" __global__

// A1: beacon messages
DG_KERNEL void __launch_bounds__(256) k_beacon_msgs(uint32_t n, const uint64_t* prev_round, const uint64_t* round,
                                                    const uint8_t* prev_sigs, const uint32_t* off, uint8_t* out32) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t a = off[i], b = off[i + 1];
  beacon_message(out32 + 32ull * i, prev_sigs + a, b - a, prev_round[i], round[i]);
}

// A2: randomness
DG_KERNEL void __launch_bounds__(256) k_randomness(uint32_t n, const uint8_t* sigs96, uint8_t* out32) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  Sha256 s;
  sha256_init(s);
  sha256_update(s, sigs96 + 96ull * i, 96);
  sha256_final(s, out32 + 32ull * i);
}

// A13: link check
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

// A9: full hash-to-G2, compressed
DG_KERNEL void __launch_bounds__(128) k_hash_to_g2(uint32_t n, const uint8_t* msgs, uint32_t msg_len,
                                                   const uint8_t* dst, uint32_t dst_len, uint8_t* out96) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  G2J h = hash_to_g2(msgs + (size_t)msg_len * i, msg_len, dst, dst_len);
  g2_compress_aff(out96 + 96ull * i, g2_to_aff(h));
}

// hash-to-curve without cofactor clearing (RLC path)
DG_KERNEL void __launch_bounds__(128) k_h2c_uncleared(uint32_t n, const uint8_t* msgs, uint32_t msg_len,
                                                      const uint8_t* dst, uint32_t dst_len, G2JStore* outQ) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  store_g2j(outQ[i], hash_to_g2_uncleared(msgs + (size_t)msg_len * i, msg_len, dst, dst_len));
}

// sigma decode + subgroup check (A10)
DG_KERNEL void __launch_bounds__(128) k_decode_sigs(uint32_t n, const uint8_t* sigs, uint32_t stride, uint32_t offset,
                                                    G2AStore* outS, uint8_t* status) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  G2A a;
  bool ok = g2_decompress(a, sigs + (size_t)stride * i + offset, true);
  if (!ok) a = G2A{fp2_zero(), fp2_zero(), true};
  store_g2a(outS[i], a);
  status[i] = ok ? DG_ST_OK_ : DG_ST_SIG_DECODE_;
}

// G1 decode (keys, commits), with subgroup check
DG_KERNEL void __launch_bounds__(64) k_decode_g1(uint32_t n, const uint8_t* in48, G1AStore* out, uint8_t* status) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  G1A a;
  bool ok = g1_decompress(a, in48 + 48ull * i, true);
  if (!ok) a = G1A{fp_zero(), fp_zero(), true};
  store_g1a(out[i], a);
  status[i] = ok ? DG_ST_OK_ : DG_ST_PK_DECODE_;
}

// RLC scaling: R_i = rho_i Q_i, T_i = rho_i S_i (O for items whose sigma did not decode)
DG_KERNEL void __launch_bounds__(128) k_rlc_scale(uint32_t n, uint64_t seed, const G2JStore* Q, const G2AStore* S,
                                                  const uint8_t* status, G2JStore* R, G2JStore* T) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  if (status[i] != DG_ST_OK_) {
    store_g2j(R[i], jac_infinity<Fp2>());
    store_g2j(T[i], jac_infinity<Fp2>());
    return;
  }
  uint64_t rho = rlc_coeff(seed, i);
  store_g2j(R[i], jac_mul_u64(load_g2j(Q[i]), rho));
  store_g2j(T[i], jac_mul_u64(jac_from_aff(load_g2a(S[i])), rho));
}

// out[j] = sum of in[j*chunk .. min(n, (j+1)*chunk))
DG_KERNEL void __launch_bounds__(128) k_sum_points(uint32_t n, uint32_t chunk, const G2JStore* in, G2JStore* out) {
  uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t a = j * chunk;
  if (a >= n) return;
  uint32_t b = a + chunk < n ? a + chunk : n;
  G2J acc = load_g2j(in[a]);
  for (uint32_t k = a + 1; k < b; ++k) acc = jac_add(acc, load_g2j(in[k]));
  store_g2j(out[j], acc);
}

// batch verdict: e(pk, h_eff * sumR) * e(-g1, sumT) == 1   -> *ok = 1/0
DG_KERNEL void __launch_bounds__(64) k_rlc_final(const G1AStore* pk, const G2JStore* sumR, const G2JStore* sumT,
                                                 uint32_t* ok) {
  if (blockIdx.x != 0 || threadIdx.x != 0) return;
  G1A P[2];
  G2A Q[2];
  int np = 0;
  G1A key = load_g1a(pk[0]);
  G2A a = g2_to_aff(g2_clear_cofactor(load_g2j(sumR[0])));
  G2A b = g2_to_aff(load_g2j(sumT[0]));
  if (!key.inf && !a.inf) {
    P[np] = key;
    Q[np] = a;
    ++np;
  }
  if (!b.inf) {
    P[np] = G1A{fp_const(G1_GEN_X), fp_const(G1_GEN_NEG_Y), false};
    Q[np] = b;
    ++np;
  }
  bool good = np == 0 ? true : fp12_is_one(final_exp_cubed(miller_loop<2>(P, Q, np)));
  *ok = good ? 1u : 0u;
}

// per-item bls.Verify with precomputed uncleared hash Q_i and decoded S_i; pk index per item (or 0)
DG_KERNEL void __launch_bounds__(64) k_verify_items(uint32_t n, const G1AStore* pks, const uint32_t* pk_idx,
                                                    const G2JStore* Q, const uint32_t* q_idx, const G2AStore* S,
                                                    uint8_t* status) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  if (status[i] != DG_ST_OK_) return;
  G1A key = load_g1a(pks[pk_idx ? pk_idx[i] : 0]);
  G2A h = g2_to_aff(g2_clear_cofactor(load_g2j(Q[q_idx ? q_idx[i] : i])));
  G2A s = load_g2a(S[i]);
  G1A P[2];
  G2A Qa[2];
  int np = 0;
  if (!key.inf && !h.inf) {
    P[np] = key;
    Qa[np] = h;
    ++np;
  }
  if (!s.inf) {
    P[np] = G1A{fp_const(G1_GEN_X), fp_const(G1_GEN_NEG_Y), false};
    Qa[np] = s;
    ++np;
  }
  bool good = np == 0 ? true : fp12_is_one(final_exp_cubed(miller_loop<2>(P, Qa, np)));
  status[i] = good ? DG_ST_OK_ : DG_ST_BAD_SIG_;
}
#endif

}  // namespace dg
