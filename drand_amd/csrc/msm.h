// Pippenger bucket multi-scalar multiplication on G2 for the random linear combinations of the verify
// path: T = sum_r alpha_r V_r (signature side) and, with a single key, K = sum_r alpha_r Q_r (hash side),
// both with the same 64-bit coefficients, so one bucket sort serves both sums.
//
//   window c = 8 bits, 8 windows, 255 buckets per window (digit 0 contributes nothing)
//   1. k_msm_count    histogram of (window, digit) over the active rounds
//   2. k_msm_scan     bucket offsets and per-bucket chunk offsets (one workgroup)
//   3. k_msm_scatter  round indices into bucket order (atomics: order inside a bucket is arbitrary,
//                     sums are exact group elements, so the result does not depend on it)
//   4. k_msm_chunks   each lane sums one chunk of <= MSM_CHUNK points of one bucket
//   5. k_msm_buckets  each lane sums the chunks of one bucket
//   6. k_msm_groups   running sums over groups of 17 buckets: sum_b (b - lo + 1) B_b + (lo - 1) sum_b B_b
//   7. k_msm_windows  per window: sum of its groups, times 2^(8w); then the 8 window terms are summed
// Work: 8 bucket additions per point instead of a 64-bit double-and-add (64 doublings + 64 divergent
// additions) per point.
#pragma once
// included from kernels.h (uses rlc_alpha, the G2JStore layout and jac_mul_small defined there)

namespace dg {

constexpr uint32_t MSM_C = 8, MSM_WIN = 8, MSM_NB = 256, MSM_NBK = MSM_WIN * MSM_NB;  // 2048 bucket slots
constexpr uint32_t MSM_CHUNK = 16;
constexpr uint32_t MSM_GROUP = 17, MSM_NGROUP = 15;  // 255 = 15 * 17 buckets per window

#if defined(__HIP__)
DG_KERNEL void __launch_bounds__(256) k_msm_count(uint32_t R, uint64_t seed, const uint8_t* active, uint32_t* count) {
  uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= R || !active[r]) return;
  uint64_t a = rlc_alpha(seed, r);
  for (uint32_t w = 0; w < MSM_WIN; ++w) {
    uint32_t d = (uint32_t)(a >> (MSM_C * w)) & (MSM_NB - 1);
    if (d) atomicAdd(&count[w * MSM_NB + d], 1u);
  }
}

// offset[b] = exclusive scan of count; cursor = offset; chunk_off[b] = exclusive scan of ceil(count/CHUNK),
// chunk_off[MSM_NBK] = total chunks.  One workgroup of 256 lanes, 8 slots each.
DG_KERNEL void __launch_bounds__(256) k_msm_scan(const uint32_t* count, uint32_t* offset, uint32_t* cursor,
                                                 uint32_t* chunk_off) {
  __shared__ uint32_t s_cnt[256], s_chk[256];
  const uint32_t t = threadIdx.x;
  uint32_t c = 0, k = 0;
  for (uint32_t j = 0; j < 8; ++j) {
    uint32_t v = count[t * 8 + j];
    c += v;
    k += (v + MSM_CHUNK - 1) / MSM_CHUNK;
  }
  s_cnt[t] = c;
  s_chk[t] = k;
  __syncthreads();
  if (t == 0) {
    uint32_t a = 0, b = 0;
    for (uint32_t i = 0; i < 256; ++i) {
      uint32_t x = s_cnt[i], y = s_chk[i];
      s_cnt[i] = a;
      s_chk[i] = b;
      a += x;
      b += y;
    }
    chunk_off[MSM_NBK] = b;
  }
  __syncthreads();
  uint32_t a = s_cnt[t], b = s_chk[t];
  for (uint32_t j = 0; j < 8; ++j) {
    uint32_t i = t * 8 + j, v = count[i];
    offset[i] = a;
    cursor[i] = a;
    chunk_off[i] = b;
    a += v;
    b += (v + MSM_CHUNK - 1) / MSM_CHUNK;
  }
}

DG_KERNEL void __launch_bounds__(256) k_msm_scatter(uint32_t R, uint64_t seed, const uint8_t* active, uint32_t* cursor,
                                                    uint32_t* list) {
  uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= R || !active[r]) return;
  uint64_t a = rlc_alpha(seed, r);
  for (uint32_t w = 0; w < MSM_WIN; ++w) {
    uint32_t d = (uint32_t)(a >> (MSM_C * w)) & (MSM_NB - 1);
    if (d) list[atomicAdd(&cursor[w * MSM_NB + d], 1u)] = r;
  }
}

// lane g: side = g / max_chunks, chunk c = g % max_chunks; sums its chunk of points of side `side`
// (side 0: PA, side 1: PB) into out[side * max_chunks + c]
DG_KERNEL void __launch_bounds__(128) k_msm_chunks(uint32_t max_chunks, uint32_t nsides, const uint32_t* count,
                                                   const uint32_t* offset, const uint32_t* chunk_off,
                                                   const uint32_t* list, const G2JStore* PA, const G2JStore* PB,
                                                   G2JStore* out) {
  uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= max_chunks * nsides) return;
  uint32_t side = g / max_chunks, c = g % max_chunks;
  if (c >= chunk_off[MSM_NBK]) return;
  // bucket of chunk c: last b with chunk_off[b] <= c
  uint32_t lo = 0, hi = MSM_NBK;
  while (hi - lo > 1) {
    uint32_t mid = (lo + hi) / 2;
    if (chunk_off[mid] <= c)
      lo = mid;
    else
      hi = mid;
  }
  uint32_t b = lo;
  uint32_t first = offset[b] + (c - chunk_off[b]) * MSM_CHUNK;
  uint32_t last = offset[b] + count[b];
  if (last > first + MSM_CHUNK) last = first + MSM_CHUNK;
  const G2JStore* P = side ? PB : PA;
  G2J acc = load_g2j(P[list[first]]);
  for (uint32_t i = first + 1; i < last; ++i) acc = jac_add(acc, load_g2j(P[list[i]]));
  store_g2j(out[side * max_chunks + c], acc);
}

// lane g: side = g / NBK, bucket b: B[side][b] = sum of its chunks
DG_KERNEL void __launch_bounds__(128) k_msm_buckets(uint32_t max_chunks, uint32_t nsides, const uint32_t* chunk_off,
                                                    const G2JStore* chunks, G2JStore* B) {
  uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= MSM_NBK * nsides) return;
  uint32_t side = g / MSM_NBK, b = g % MSM_NBK;
  uint32_t c0 = chunk_off[b], c1 = chunk_off[b + 1];
  G2J acc = jac_infinity<Fp2>();
  for (uint32_t c = c0; c < c1; ++c) acc = jac_add(acc, load_g2j(chunks[side * max_chunks + c]));
  store_g2j(B[g], acc);
}

// lane g: side, window w, group q over buckets lo..hi (1-based digits):
//   G = sum_{b=lo..hi} (b - lo + 1) B_b + (lo - 1) sum_{b=lo..hi} B_b = sum_b b B_b
DG_KERNEL void __launch_bounds__(64) k_msm_groups(uint32_t nsides, const G2JStore* B, G2JStore* G) {
  uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t per_side = MSM_WIN * MSM_NGROUP;
  if (g >= per_side * nsides) return;
  uint32_t side = g / per_side, w = (g % per_side) / MSM_NGROUP, q = g % MSM_NGROUP;
  uint32_t lo = 1 + q * MSM_GROUP, hi = lo + MSM_GROUP - 1;
  const G2JStore* Bw = B + side * MSM_NBK + w * MSM_NB;
  G2J run = jac_infinity<Fp2>(), acc = jac_infinity<Fp2>();
  for (uint32_t b = hi; b >= lo; --b) {
    run = jac_add(run, load_g2j(Bw[b]));
    acc = jac_add(acc, run);
  }
  if (lo > 1) acc = jac_add(acc, jac_mul_small(run, lo - 1));
  store_g2j(G[g], acc);
}

// lane g: side, window w: S_w = 2^(8w) * sum_q G[side][w][q]; then lane (side, 0) sums the 8 windows
DG_KERNEL void __launch_bounds__(64) k_msm_windows(uint32_t nsides, const G2JStore* G, G2JStore* out) {
  __shared__ G2JStore S[2 * MSM_WIN];
  uint32_t g = threadIdx.x;
  if (g < MSM_WIN * nsides) {
    uint32_t side = g / MSM_WIN, w = g % MSM_WIN;
    const G2JStore* Gw = G + side * MSM_WIN * MSM_NGROUP + w * MSM_NGROUP;
    G2J acc = load_g2j(Gw[0]);
    for (uint32_t q = 1; q < MSM_NGROUP; ++q) acc = jac_add(acc, load_g2j(Gw[q]));
    for (uint32_t k = 0; k < MSM_C * w; ++k) acc = jac_dbl(acc);
    store_g2j(S[g], acc);
  }
  __syncthreads();
  if (g < nsides) {
    G2J acc = load_g2j(S[g * MSM_WIN]);
    for (uint32_t w = 1; w < MSM_WIN; ++w) acc = jac_add(acc, load_g2j(S[g * MSM_WIN + w]));
    store_g2j(out[g], acc);
  }
}
#endif

}  // namespace dg
