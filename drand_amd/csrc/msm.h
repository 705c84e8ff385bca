// Pippenger bucket multi-scalar multiplication on G2 for the random linear combinations of the verify
// path: T = sum_r alpha_r V_r (signature side) and, with a single key, K = sum_r alpha_r Q_r (hash side),
// both with the same 64-bit coefficients, so one bucket sort serves both sums.
//
//   window c = 8 bits, 8 windows, 255 buckets per window (digit 0 contributes nothing)
//   1. k_msm_count    histogram of (window, digit) over the active rounds
//   2. k_msm_scan     bucket offsets and per-bucket chunk offsets (one workgroup)
//   3. k_msm_scatter  round indices into bucket order (atomics: order inside a bucket is arbitrary,
//                     sums are exact group elements, so the result does not depend on it)
//   4. k_msm_chunks       each lane sums one chunk of <= MSM_CHUNK points of one bucket (mixed additions
//                         for Z = 1 inputs)
//   5. k_msm_buckets      MSM_BSPLIT (32) lanes per bucket sum its chunks strided; pairwise k_sum_rows fold them
//   6. k_msm_slices       bucket aggregation by bit slices: sum_b b B_b = sum_k 2^k S_k, S_k = sum of the
//                         buckets whose digit has bit k set (16 lanes per (window, k), then k_sum_rows)
//   7. k_msm_horner_coop  per window, cooperatively (coop.h): W_w = sum_k 2^k S_k, times 2^(8w)
//   8. k_msm_final_coop   the sum of the 8 window terms
// Work: 8 bucket additions per point instead of a 64-bit double-and-add (64 doublings + 64 divergent
// additions) per point.
//
// Batched G2 subgroup check (single-key path, one item per round): with nwin = MSM_WT the signature
// side also sums MSM_TWIN "test windows" whose 8-bit digits come from an independent hash of (seed, r),
// and every window sum W_w of that side (the 8 alpha windows, whose digits are the independent bytes of
// alpha_r, and the test windows) must lie in G2 (k_msm_subgroup).  The E'(Fp2) cofactor h2 is prime to
// r and its smallest prime factor is 13, so a non-zero torsion component E_r of some sigma_r survives
// in W_w = sum_r d_{w,r} sigma_r unless d_{w,r} falls in one residue class mod ord(E_r) >= 13: at most
// 20 of the 256 digit values (10 of the 128 odd low digits of alpha) -- <= 2^-3.68 per window, 2^-66
// over 18 windows.  A failed check sends the batch to the exact per-item pass, which subgroup-checks
// each signature itself.  This replaces a 64-doubling psi check per signature by 10 bucket additions.
#pragma once
// included from kernels.h (uses rlc_alpha, the G2JStore layout and jac_mul_small defined there)

namespace dg {

constexpr uint32_t MSM_C = 8, MSM_WIN = 8, MSM_NB = 256, MSM_NBK = MSM_WIN * MSM_NB;  // 2048 bucket slots
constexpr uint32_t MSM_TWIN = 10, MSM_WT = MSM_WIN + MSM_TWIN;  // test windows of the batched subgroup check
constexpr uint32_t MSM_NBT = MSM_WT * MSM_NB;                   // 4608 bucket slots with the test windows
// keyed MSM bucket key: (window, digit, key set), the set fastest
DGI uint32_t kmsm_key(uint32_t w, uint32_t d, uint32_t set, uint32_t nsets) { return (w * MSM_NB + d) * nsets + set; }
#ifndef DG_MSM_LDS
#define DG_MSM_LDS 1  // chunk sums: 1 running sum in LDS, 2 in registers (g2_madd_lds form), 0 round-2 form
#endif
#ifndef DG_MSM_WAVES
#define DG_MSM_WAVES DG_HOT_WAVES  // min waves per SIMD of the chunk sums
#endif
constexpr uint32_t MSM_CHUNK = 8;   // points per first-level lane
// points per chunk of the keyed MSM: its buckets hold ~400 points each at C3 (100k rounds: 6.4M items x 18
// windows over 256 digits x 64 key sets), so longer mixed-addition chunks (29 Fp products per point) leave fewer
// chunk sums for the bucket lanes' full Jacobian additions (43 per chunk)
#ifndef DG_KMSM_CHUNK
#define DG_KMSM_CHUNK 32
#endif
constexpr uint32_t KMSM_CHUNK = DG_KMSM_CHUNK;
constexpr uint32_t MSM_BSPLIT = 32;  // lanes per bucket at the second level
#ifndef DG_KMSM_BSPLIT
#define DG_KMSM_BSPLIT 4
#endif
constexpr uint32_t KMSM_BSPLIT = DG_KMSM_BSPLIT;  // lanes per keyed bucket over its affine chunk sums
constexpr uint32_t MSM_SLICE_LANES = 64;  // lanes per (side, window, bit slice) in k_msm_slices

#if defined(__HIP__) && DG_TU_LIB
// digits of round r in windows 0..nwin-1: the bytes of alpha_r, then (nwin > MSM_WIN) the first
// MSM_TWIN bytes of SHA-256(seed' || r), an independent hash
struct MsmDigits {
  uint64_t a;
  uint8_t t[32];
  DGI MsmDigits(uint64_t seed, uint32_t r, uint32_t nwin) : a(rlc_alpha(seed, r)) {
    if (nwin > MSM_WIN) rlc_digest(seed ^ 0x5375626772705465ull, r, t);  // "SubgrpTe"
  }
  DGI uint32_t operator()(uint32_t w) const {
    return w < MSM_WIN ? (uint32_t)(a >> (MSM_C * w)) & (MSM_NB - 1) : (uint32_t)t[w - MSM_WIN];
  }
};

DG_KERNEL void __launch_bounds__(256) k_msm_count(uint32_t R, uint32_t nwin, const uint64_t* seedp, const uint8_t* active,
                                                  uint32_t* count) {
  const uint64_t seed = *seedp;
  uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= R || !active[r]) return;
  const MsmDigits dg(seed, r, nwin);
  for (uint32_t w = 0; w < nwin; ++w) {
    uint32_t d = dg(w);
    if (d) atomicAdd(&count[w * MSM_NB + d], 1u);
  }
}

// offset[b] = exclusive scan of count; cursor = offset; chunk_off[b] = exclusive scan of ceil(count/CHUNK),
// chunk_off[nbk] = total chunks.  One workgroup of 256 lanes, nbk / 256 (= nwin) slots each.
DG_KERNEL void __launch_bounds__(256) k_msm_scan(uint32_t nbk, const uint32_t* count, uint32_t* offset,
                                                 uint32_t* cursor, uint32_t* chunk_off) {
  __shared__ uint32_t s_cnt[256], s_chk[256];
  const uint32_t t = threadIdx.x, per = nbk / 256;
  uint32_t c = 0, k = 0;
  for (uint32_t j = 0; j < per; ++j) {
    uint32_t v = count[t * per + j];
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
    chunk_off[nbk] = b;
  }
  __syncthreads();
  uint32_t a = s_cnt[t], b = s_chk[t];
  for (uint32_t j = 0; j < per; ++j) {
    uint32_t i = t * per + j, v = count[i];
    offset[i] = a;
    cursor[i] = a;
    chunk_off[i] = b;
    a += v;
    b += (v + MSM_CHUNK - 1) / MSM_CHUNK;
  }
}

DG_KERNEL void __launch_bounds__(256) k_msm_scatter(uint32_t R, uint32_t nwin, const uint64_t* seedp, const uint8_t* active,
                                                    uint32_t* cursor, uint32_t* list) {
  const uint64_t seed = *seedp;
  uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= R || !active[r]) return;
  const MsmDigits dg(seed, r, nwin);
  for (uint32_t w = 0; w < nwin; ++w) {
    uint32_t d = dg(w);
    if (d) list[atomicAdd(&cursor[w * MSM_NB + d], 1u)] = r;
  }
}

#endif

// the chunk sums are the MSM's bulk work: hot translation unit (kernels_hot.hip, flat, 2 waves/SIMD)
#if defined(__HIP__) && DG_TU_HOT
// lane g: side = g / max_chunks, chunk c = g % max_chunks; sums its chunk of points of side `side`
// (side 0: PA, side 1: PB) into out[side * max_chunks + c]; side 1 has no test windows (buckets >= MSM_NBK)
DG_KERNEL void __launch_bounds__(128, DG_MSM_WAVES) k_msm_chunks(uint32_t max_chunks, uint32_t nsides, uint32_t nbk, const uint32_t* count,
                                                   const uint32_t* offset, const uint32_t* chunk_off,
                                                   const uint32_t* list, const G2JStore* PA, const G2JStore* PB,
                                                   G2JStore* out) {
  uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= max_chunks * nsides) return;
  uint32_t side = g / max_chunks, c = g % max_chunks;
  if (c >= chunk_off[side ? MSM_NBK : nbk]) return;
  // bucket of chunk c: last b with chunk_off[b] <= c
  uint32_t lo = 0, hi = nbk;
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
  const Fp2 one = fp2_one();
#if DG_MSM_LDS
  // the running sum lives in LDS (36 KB per workgroup, 4 workgroups per CU at 2 waves/SIMD) or in registers
#if DG_MSM_LDS == 1
  __shared__ G2JStore s_acc[128];
  G2JStore& acc = s_acc[threadIdx.x];
#else
  G2JStore acc;
#endif
  acc = P[list[first]];
  for (uint32_t i = first + 1; i < last; ++i) {
    const G2JStore& q = P[list[i]];
    if (fp2_eq(q.z, one))
      g2_madd_lds(acc, q.x, q.y);
    else if (!fp2_is_zero(q.z))
      store_g2j(acc, g2_add_rare(load_g2j(acc), load_g2j(q)));
  }
  out[side * max_chunks + c] = acc;
#else
  G2J acc = load_g2j(P[list[first]]);
  for (uint32_t i = first + 1; i < last; ++i) {
    const G2JStore& q = P[list[i]];
    // signatures and hashes enter normalised (Z = 1) or as the identity (Z = 0): mixed additions (7M + 4S
    // instead of 11M + 5S in Fp2); any other Z takes the full addition, out of line
    if (fp2_eq(q.z, one))
      acc = g2_madd_lean(acc, q.x, q.y);
    else if (!fp2_is_zero(q.z))
      acc = g2_add_rare(acc, load_g2j(q));
  }
  store_g2j(out[side * max_chunks + c], acc);
#endif
}

#elif defined(__HIP__)
DG_KERNEL void __launch_bounds__(128, DG_MSM_WAVES) k_msm_chunks(uint32_t max_chunks, uint32_t nsides, uint32_t nbk, const uint32_t* count,
                                                   const uint32_t* offset, const uint32_t* chunk_off,
                                                   const uint32_t* list, const G2JStore* PA, const G2JStore* PB,
                                                   G2JStore* out);
#endif

// ---------------------------------------------------------------------------------------------------
// Affine first levels (single-key path, every input point with Z = 1 or Z = 0).  Instead of one lane summing
// a chunk of 8 points with mixed Jacobian additions (7M + 4S in Fp2 each, 29 Fp products), the points of every
// bucket are summed pairwise in MSM_AFF_L levels of affine additions, each level's denominators inverted
// together (Montgomery's trick over the whole batch, batch_inv):
//   lambda = (y2 - y1) / (x2 - x1), x3 = lambda^2 - x1 - x2, y3 = lambda (x1 - x3) - y1
// 1/d = conj(d) / N(d) with N(d) = d0^2 + d1^2 in Fp, so one Fp inversion per level serves every pair: about
// 2 (norm) + 3 (batch inversion) + 2 (conj) + 8 (lambda, x3, y3) = 15 Fp products per addition.
// Level l pairs the entries i and i + 2^l of each group of 2^(l+1) consecutive entries of a bucket (bucket order of
// the shared list) and writes the sum in place at i (A: one G2AStore per list position and side); after
// MSM_AFF_L levels A[offset[b] + k 2^L] holds the k-th chunk sum of bucket b, which k_msm_buckets_aff reads.
// Exceptional pairs are exact: P + (-P) = identity, P + P by the tangent (d = 2y; E' has no 2-torsion, h2 is
// odd), identity operands pass the other one through; they take no inversion (denominator 1).
#ifndef DG_MSM_AFF_L
#define DG_MSM_AFF_L 3
#endif
constexpr uint32_t MSM_AFF_L = DG_MSM_AFF_L;  // affine levels: chunk sums of 2^3 = 8 entries (A/B: DG_MSM_AFF_L)
DGI G2A aff_src0(const G2JStore& p) { return G2A{p.x, p.y, fp_is_zero(p.z.c0)}; }  // Z is 0 or 1 (checked below)
// msm_run's precondition for the affine levels: every input point has Z = 0 (identity) or Z = 1.  Level 0 checks
// it on every entry it reads and raises *bad otherwise: the caller's batch equation then fails and every item
// takes its own exact check, so a Jacobian input can never be summed wrong silently.
DGI bool aff_input_ok(const G2JStore& p) { return fp2_is_zero(p.z) || fp2_eq(p.z, fp2_one()); }
DGI G2A aff_srcA(const G2AStore& p) { return G2A{p.x, p.y, p.inf != 0}; }
// group g of level l (groups of 2^(l+1) entries of one bucket) -> its first entry i and bucket end
DGI bool aff_group(uint32_t nbk, const uint32_t* count, const uint32_t* offset, const uint32_t* gofs, uint32_t l,
                   uint32_t g, uint32_t& i, uint32_t& end) {
  uint32_t lo = 0, hi = nbk;
  while (hi - lo > 1) {
    uint32_t mid = (lo + hi) / 2;
    if (gofs[mid] <= g)
      lo = mid;
    else
      hi = mid;
  }
  i = offset[lo] + ((g - gofs[lo]) << (l + 1));
  end = offset[lo] + count[lo];
  return i + (1u << l) < end;  // has a partner
}

#if defined(__HIP__) && DG_TU_LIB
// offset / cursor as k_msm_scan, and gofs[l * (nbk + 1) + b] = exclusive scan of ceil(count / 2^(l+1)) for the
// MSM_AFF_L levels (gofs[l * (nbk + 1) + nbk] = groups of level l).  One workgroup of 256 lanes.
DG_KERNEL void __launch_bounds__(256) k_msm_scan_aff(uint32_t nbk, const uint32_t* count, uint32_t* offset,
                                                     uint32_t* cursor, uint32_t* gofs) {
  __shared__ uint32_t s_cnt[256], s_g[MSM_AFF_L][256];
  const uint32_t t = threadIdx.x, per = nbk / 256;
  uint32_t c = 0, k[MSM_AFF_L] = {};
  for (uint32_t j = 0; j < per; ++j) {
    uint32_t v = count[t * per + j];
    c += v;
    for (uint32_t l = 0; l < MSM_AFF_L; ++l) k[l] += (v + (2u << l) - 1) >> (l + 1);
  }
  s_cnt[t] = c;
  for (uint32_t l = 0; l < MSM_AFF_L; ++l) s_g[l][t] = k[l];
  __syncthreads();
  if (t <= MSM_AFF_L) {  // lane 0: the entry scan, lane 1 + l: level l's group scan
    uint32_t* s = t == 0 ? s_cnt : s_g[t - 1];
    uint32_t a = 0;
    for (uint32_t i = 0; i < 256; ++i) {
      uint32_t x = s[i];
      s[i] = a;
      a += x;
    }
    if (t > 0) gofs[(t - 1) * (nbk + 1) + nbk] = a;
  }
  __syncthreads();
  uint32_t a = s_cnt[t], b[MSM_AFF_L];
  for (uint32_t l = 0; l < MSM_AFF_L; ++l) b[l] = s_g[l][t];
  for (uint32_t j = 0; j < per; ++j) {
    uint32_t i = t * per + j, v = count[i];
    offset[i] = a;
    cursor[i] = a;
    a += v;
    for (uint32_t l = 0; l < MSM_AFF_L; ++l) {
      gofs[l * (nbk + 1) + i] = b[l];
      b[l] += (v + (2u << l) - 1) >> (l + 1);
    }
  }
}
#endif

#if defined(__HIP__) && DG_TU_HOT
// level l, lane t = side * maxg + g: the norm of the denominator of group g's pair (1 where no inversion is
// needed, and on the lanes past the level's group count, so every value batch_inv sees is a field element)
DG_KERNEL void __launch_bounds__(128) k_msm_aff_den(uint32_t l, uint32_t maxg, uint32_t nsides, uint32_t nbk,
                                                    const uint32_t* count, const uint32_t* offset, const uint32_t* gofs,
                                                    const uint32_t* list, const G2JStore* PA, const G2JStore* PB,
                                                    const G2AStore* A, uint32_t E, Fp* den) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= maxg * nsides) return;
  const uint32_t side = t / maxg, g = t % maxg;
  Fp n = fp_one();
  uint32_t i, end;
  if (g < gofs[side ? MSM_NBK : nbk] && aff_group(nbk, count, offset, gofs, l, g, i, end)) {
    // read only what the norm needs: the identity flags and x (y only for equal x)
    const uint32_t j = i + (1u << l);
    const Fp2 *px, *py, *qx, *qy;
    bool pinf, qinf;
    if (l == 0) {
      const G2JStore* P = side ? PB : PA;
      const G2JStore &a = P[list[i]], &b = P[list[j]];
      pinf = fp_is_zero(a.z.c0);  // Z is 0 or 1 (msm_run's precondition)
      qinf = fp_is_zero(b.z.c0);
      px = &a.x, py = &a.y, qx = &b.x, qy = &b.y;
    } else {
      const G2AStore &a = A[(size_t)side * E + i], &b = A[(size_t)side * E + j];
      pinf = a.inf != 0;
      qinf = b.inf != 0;
      px = &a.x, py = &a.y, qx = &b.x, qy = &b.y;
    }
    if (!pinf && !qinf) {
      const Fp2 x1 = *px, x2 = *qx;
      if (!fp2_eq(x1, x2))
        n = fp2_norm(fp2_sub(x2, x1));
      else if (fp2_eq(*py, *qy))
        n = fp2_norm(fp2_dbl(*py));  // the same as g2_aff_den for kinds 1 and 2
    }
  }
  den[t] = n;
}

// level l: the pair sums with the inverted norms (same lanes as k_msm_aff_den); level 0 also copies the unpaired
// entries into A
DG_KERNEL void __launch_bounds__(128, DG_HOT_WAVES) k_msm_aff_add(uint32_t l, uint32_t maxg, uint32_t nsides,
                                                                 uint32_t nbk, const uint32_t* count,
                                                                 const uint32_t* offset, const uint32_t* gofs,
                                                                 const uint32_t* list, const G2JStore* PA,
                                                                 const G2JStore* PB, G2AStore* A, uint32_t E,
                                                                 const Fp* ninv, uint32_t* bad) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= maxg * nsides) return;
  const uint32_t side = t / maxg, g = t % maxg;
  if (g >= gofs[side ? MSM_NBK : nbk]) return;
  uint32_t i, end;
  const bool pair = aff_group(nbk, count, offset, gofs, l, g, i, end);
  G2AStore* Aside = A + (size_t)side * E;
  if (!pair && l > 0) return;  // the lone entry already sits at i
  G2A p, q;
  if (l == 0) {
    const G2JStore* P = side ? PB : PA;
    const G2JStore& a = P[list[i]];
    if (!aff_input_ok(a)) atomicOr(bad, 1u);
    p = aff_src0(a);
    if (!pair) {
      store_g2a(Aside[i], p);
      return;
    }
    const G2JStore& b = P[list[i + 1]];
    if (!aff_input_ok(b)) atomicOr(bad, 1u);
    q = aff_src0(b);
  } else {
    p = aff_srcA(Aside[i]);
    q = aff_srcA(Aside[i + (1u << l)]);
  }
  const G2A r = g2_aff_sum(p, q, g2_aff_kind(p, q), ninv[t]);
  store_g2a(Aside[i], r);
}

#elif defined(__HIP__)
DG_KERNEL void __launch_bounds__(128) k_msm_aff_den(uint32_t l, uint32_t maxg, uint32_t nsides, uint32_t nbk,
                                                    const uint32_t* count, const uint32_t* offset, const uint32_t* gofs,
                                                    const uint32_t* list, const G2JStore* PA, const G2JStore* PB,
                                                    const G2AStore* A, uint32_t E, Fp* den);
DG_KERNEL void __launch_bounds__(128, DG_HOT_WAVES) k_msm_aff_add(uint32_t l, uint32_t maxg, uint32_t nsides,
                                                                 uint32_t nbk, const uint32_t* count,
                                                                 const uint32_t* offset, const uint32_t* gofs,
                                                                 const uint32_t* list, const G2JStore* PA,
                                                                 const G2JStore* PB, G2AStore* A, uint32_t E,
                                                                 const Fp* ninv, uint32_t* bad);
#endif

// 2-D segmented sum: out[row * ocols + j] = sum_{c in [j*chunk, (j+1)*chunk) and < cols} in[row * cols + c]
// (rows of a block with skip[row / 64] != 0 are left alone: skip may be null).  Hot TU: the running sum in LDS and
// the additions inlined with serialised products (curve.h g2_add_lds), no call frames -- these launches sit on a
// batch's critical path (11 per headline batch), where the library TU's out-of-line products cost ~180 us each.
#if defined(__HIP__) && DG_TU_HOT
DG_KERNEL void __launch_bounds__(128, DG_MSM_WAVES) k_sum_rows(uint32_t rows, uint32_t cols, uint32_t chunk,
                                                                const G2JStore* in, G2JStore* out, const uint8_t* skip) {
  DG_HI();
  __shared__ G2JStore s_acc[128];
  uint32_t ocols = (cols + chunk - 1) / chunk;
  uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= rows * ocols) return;
  uint32_t row = g / ocols, j = g % ocols;
  if (skip && skip[row / 64]) return;
  uint32_t a = j * chunk, b = a + chunk < cols ? a + chunk : cols;
  const G2JStore* p = in + (size_t)row * cols;
  G2JStore& acc = s_acc[threadIdx.x];
  acc = p[a];
  for (uint32_t c = a + 1; c < b; ++c) g2_add_lds(acc, load_g2j(p[c]));
  out[g] = acc;
}
#elif defined(__HIP__)
DG_KERNEL void __launch_bounds__(128, DG_MSM_WAVES) k_sum_rows(uint32_t rows, uint32_t cols, uint32_t chunk,
                                                                const G2JStore* in, G2JStore* out, const uint8_t* skip);
#endif

// the bucket sums from the affine chunk sums: lane (side, b, q < bsplit) adds chunks q, q + bsplit, ... of bucket b
// (A[offset[b] + c 2^L]) with mixed additions, the running sum in LDS (g2_madd_lds); the bsplit partials
// BP[sb * bsplit + q] are then row-summed (bsplit <= MSM_BSPLIT, a power of two)
#if defined(__HIP__) && DG_TU_HOT
DG_KERNEL void __launch_bounds__(128, DG_MSM_WAVES) k_msm_buckets_aff(uint32_t nsides, uint32_t nbk, uint32_t bsplit,
                                                                      const uint32_t* count, const uint32_t* offset,
                                                                      const G2AStore* A, uint32_t E, G2JStore* BP) {
  uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= nbk * bsplit * nsides) return;
  uint32_t q = g % bsplit, sb = g / bsplit;
  uint32_t side = sb / nbk, b = sb % nbk;
  const uint32_t nch = side && b >= MSM_NBK ? 0u : (count[b] + (1u << MSM_AFF_L) - 1) >> MSM_AFF_L;
  const G2AStore* As = A + (size_t)side * E + offset[b];
  __shared__ G2JStore s_acc[128];
  G2JStore& acc = s_acc[threadIdx.x];
  store_g2j(acc, jac_infinity<Fp2>());
  for (uint32_t c = q; c < nch; c += bsplit) {
    const G2AStore& a = As[c << MSM_AFF_L];
    if (!a.inf) g2_madd_lds(acc, a.x, a.y);
  }
  BP[g] = acc;
}
#elif defined(__HIP__)
DG_KERNEL void __launch_bounds__(128, DG_MSM_WAVES) k_msm_buckets_aff(uint32_t nsides, uint32_t nbk, uint32_t bsplit,
                                                                      const uint32_t* count, const uint32_t* offset,
                                                                      const G2AStore* A, uint32_t E, G2JStore* BP);
#endif

#if defined(__HIP__) && DG_TU_LIB
// lane g: side, bucket b, lane-in-bucket q < MSM_BSPLIT: strided partial sum of the bucket's chunks,
// BP[(side * NBK + b) * MSM_BSPLIT + q]; the MSM_BSPLIT partials are then row-summed into B[side][b]
DG_KERNEL void __launch_bounds__(128, DG_BULK_WAVES) k_msm_buckets(uint32_t max_chunks, uint32_t nsides, uint32_t nbk,
                                                                   const uint32_t* chunk_off, const G2JStore* chunks,
                                                                   G2JStore* BP) {
  uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= nbk * MSM_BSPLIT * nsides) return;
  uint32_t q = g % MSM_BSPLIT, sb = g / MSM_BSPLIT;
  uint32_t side = sb / nbk, b = sb % nbk;
  uint32_t c0 = chunk_off[b], c1 = side && b >= MSM_NBK ? c0 : chunk_off[b + 1];
  G2J acc = jac_infinity<Fp2>();
  for (uint32_t c = c0 + q; c < c1; c += MSM_BSPLIT) acc = jac_add(acc, load_g2j(chunks[side * max_chunks + c]));
  store_g2j(BP[g], acc);
}

// Bucket aggregation by bit slices: sum_b b B_b = sum_k 2^k S_k with S_k = sum of the buckets whose
// digit b has bit k set (128 of the 255).  Level 1: lane (side, w, k, c < MSM_SLICE_LANES) sums 2 of those
// buckets; the pairwise row sums that follow keep the dependent-addition depth at 1 + log2(lanes).
DG_KERNEL void __launch_bounds__(128, DG_BULK_WAVES) k_msm_slices(uint32_t nsides, uint32_t nwin, const G2JStore* B,
                                                                  G2JStore* P1) {
  constexpr uint32_t L = MSM_SLICE_LANES, PER = 128 / MSM_SLICE_LANES;
  uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= nsides * nwin * MSM_C * L) return;
  uint32_t c = g % L, k = (g / L) % MSM_C, w = (g / (L * MSM_C)) % nwin, side = g / (L * MSM_C * nwin);
  const G2JStore* Bw = B + (side * nwin + w) * MSM_NB;
  G2J acc = jac_infinity<Fp2>();
  for (uint32_t i = PER * c; i < (side && w >= MSM_WIN ? 0 : PER * c + PER); ++i) {
    // i-th digit in 0..255 with bit k set: insert a 1 at bit k of i
    uint32_t b = ((i >> k) << (k + 1)) | (1u << k) | (i & ((1u << k) - 1));
    acc = jac_add(acc, load_g2j(Bw[b]));
  }
  store_g2j(P1[g], acc);
}

// one 128-lane workgroup per (side, window): W_w = sum_k 2^k S_{w,k} (Horner with cooperative doublings
// and additions, coop.h), then 2^(8w) W_w (alpha windows; test windows stay unshifted and exist only on
// the first `tsides` sides)
DG_KERNEL void __launch_bounds__(128, DG_COOP_WAVES) k_msm_horner_coop(uint32_t nwin, uint32_t tsides, const G2JStore* S,
                                                                       G2JStore* Wout) {
  DG_HI();
  __shared__ CoG2Tmp tmp;
  __shared__ CoG2 acc, nxt;
  const uint32_t sw = blockIdx.x, w = sw % nwin;
  if (sw / nwin >= tsides && w >= MSM_WIN) return;
  const G2JStore* Sw = S + sw * MSM_C;
  CO_SERIAL({
    G2J a = load_g2j(Sw[MSM_C - 1]);
    acc = CoG2{a.x, a.y, a.z};
  });
  for (int k = MSM_C - 2; k >= 0; --k) {
    co_g2_dbl(&acc, &tmp);
    CO_SERIAL({
      G2J a = load_g2j(Sw[k]);
      nxt = CoG2{a.x, a.y, a.z};
    });
    co_g2_add(&acc, &acc, &nxt, &tmp);
  }
  for (uint32_t d = 0; d < (w < MSM_WIN ? MSM_C * w : 0u); ++d) co_g2_dbl(&acc, &tmp);
  CO_SERIAL(store_g2j(Wout[sw], G2J{acc.x, acc.y, acc.z}));
}

// one 128-lane workgroup per side: out[side] = sum_{w < MSM_WIN} W[side][w]
DG_KERNEL void __launch_bounds__(128, DG_COOP_WAVES) k_msm_final_coop(uint32_t nwin, const G2JStore* W, G2JStore* out) {
  DG_HI();
  __shared__ CoG2Tmp tmp;
  __shared__ CoG2 acc, nxt;
  const uint32_t side = blockIdx.x;
  CO_SERIAL({
    G2J a = load_g2j(W[side * nwin]);
    acc = CoG2{a.x, a.y, a.z};
  });
  for (uint32_t w = 1; w < MSM_WIN; ++w) {
    CO_SERIAL({
      G2J a = load_g2j(W[side * nwin + w]);
      nxt = CoG2{a.x, a.y, a.z};
    });
    co_g2_add(&acc, &acc, &nxt, &tmp);
  }
  CO_SERIAL(store_g2j(out[side], G2J{acc.x, acc.y, acc.z}));
}

// (the batched subgroup check -- one 128-lane workgroup per window sum W[w] testing psi(P) == [z]P cooperatively,
// coop.h co_subgroup_check -- runs as extra workgroups of the Miller launch, k_pair_miller_coop; a failure sets the
// batch's flag[2], which k_final_coop folds into its verdict, so the isolation pass runs)

// ---------------------------------------------------------------------------------------------------
// Keyed MSM for the multi-key batch (VerifyPartial / Recover): T_s = sum over the batch items i of key
// slot s of alpha_{r(i)} S_i, for every slot at once.  Bucket key = (window, digit, set) with the set
// (the item's key slot) fastest, so one bucket sort serves all sets.  Then T = sum_s beta_s T_s -- the
// same alpha_r beta_s item coefficients as before, without a 64-bit scalar multiplication per item.
//   k_kmsm_count / k_kscan_* / k_kmsm_scatter   bucket sort of the item indices (multi-block scan)
//   k_kmsm_chunks                               chunk sums of <= MSM_CHUNK affine signatures
//   k_kmsm_buckets                              one lane per bucket sums its chunks
//   k_kmsm_slices                               bit-slice partials per (set, window, bit)
//   k_msm_horner_coop / k_msm_final_coop        per (set, window) / per set, as above
//   k_kmsm_beta                                 beta_s T_s, then a row sum
constexpr uint32_t KSCAN_B = 1024;  // keys per scan block


DG_KERNEL void __launch_bounds__(256) k_kmsm_count(uint32_t N, uint32_t k, uint32_t nsets, uint32_t nwin, const uint64_t* seedp,
                                                   const uint32_t* item_slot, const uint8_t* status,
                                                   const uint8_t* isolate, uint32_t* count) {
  const uint64_t seed = *seedp;
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= N || status[i] != DG_ST_OK_ || isolate[i]) return;
  const MsmDigits dg(seed, i / k, nwin);
  uint32_t s = item_slot[i];
  for (uint32_t w = 0; w < nwin; ++w) {
    uint32_t d = dg(w);
    if (d) atomicAdd(&count[kmsm_key(w, d, s, nsets)], 1u);
  }
}

// block b of KSCAN_B keys: exclusive scans of count and of ceil(count / KMSM_CHUNK) within the block,
// block totals into tot[b], tot[nblocks + b]
// (div: the chunk length of chunk_off -- KMSM_CHUNK for the Jacobian chunk sums, 2^(l+1) for the groups of affine
// level l)
DG_KERNEL void __launch_bounds__(256) k_kscan_local(uint32_t nkeys, uint32_t div, const uint32_t* count, uint32_t* offset,
                                                    uint32_t* chunk_off, uint32_t* tot) {
  __shared__ uint32_t s_c[256], s_k[256];
  const uint32_t t = threadIdx.x, base = blockIdx.x * KSCAN_B + t * 4;
  uint32_t c[4], kk[4], sc = 0, sk = 0;
  for (int j = 0; j < 4; ++j) {
    uint32_t v = base + j < nkeys ? count[base + j] : 0u;
    c[j] = sc;
    kk[j] = sk;
    sc += v;
    sk += (v + div - 1) / div;
  }
  s_c[t] = sc;
  s_k[t] = sk;
  __syncthreads();
  for (uint32_t o = 1; o < 256; o <<= 1) {  // Hillis-Steele inclusive scan
    uint32_t a = t >= o ? s_c[t - o] : 0u, b = t >= o ? s_k[t - o] : 0u;
    __syncthreads();
    s_c[t] += a;
    s_k[t] += b;
    __syncthreads();
  }
  const uint32_t pc = t ? s_c[t - 1] : 0u, pk = t ? s_k[t - 1] : 0u;
  for (int j = 0; j < 4; ++j)
    if (base + j < nkeys) {
      offset[base + j] = pc + c[j];
      chunk_off[base + j] = pk + kk[j];
    }
  if (t == 255) {
    tot[blockIdx.x] = s_c[255];
    tot[gridDim.x + blockIdx.x] = s_k[255];
  }
}
// one workgroup: exclusive scan of the nblocks block totals (in place), grand totals to chunk_off[nkeys]
DG_KERNEL void __launch_bounds__(64) k_kscan_top(uint32_t nblocks, uint32_t nkeys, uint32_t* tot, uint32_t* chunk_off) {
  if (threadIdx.x != 0) return;
  uint32_t a = 0, b = 0;
  for (uint32_t i = 0; i < nblocks; ++i) {
    uint32_t x = tot[i], y = tot[nblocks + i];
    tot[i] = a;
    tot[nblocks + i] = b;
    a += x;
    b += y;
  }
  chunk_off[nkeys] = b;
}
DG_KERNEL void __launch_bounds__(256) k_kscan_add(uint32_t nkeys, const uint32_t* tot, uint32_t* offset,
                                                  uint32_t* cursor, uint32_t* chunk_off) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nkeys) return;
  uint32_t b = i / KSCAN_B, nblocks = (nkeys + KSCAN_B - 1) / KSCAN_B;
  offset[i] += tot[b];
  cursor[i] = offset[i];
  chunk_off[i] += tot[nblocks + b];
}

DG_KERNEL void __launch_bounds__(256) k_kmsm_scatter(uint32_t N, uint32_t k, uint32_t nsets, uint32_t nwin, const uint64_t* seedp,
                                                     const uint32_t* item_slot, const uint8_t* status,
                                                     const uint8_t* isolate, uint32_t* cursor, uint32_t* list) {
  const uint64_t seed = *seedp;
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= N || status[i] != DG_ST_OK_ || isolate[i]) return;
  const MsmDigits dg(seed, i / k, nwin);
  uint32_t s = item_slot[i];
  for (uint32_t w = 0; w < nwin; ++w) {
    uint32_t d = dg(w);
    if (d) list[atomicAdd(&cursor[kmsm_key(w, d, s, nsets)], 1u)] = i;
  }
}

// lane c: the c-th chunk (<= KMSM_CHUNK affine points of one bucket)
#endif
// hot translation unit (kernels_hot.hip: flat, 2 waves/SIMD; measured -27% / -36%)
#if defined(__HIP__) && DG_TU_HOT
DG_KERNEL void __launch_bounds__(128, DG_MSM_WAVES) k_kmsm_chunks(uint32_t max_chunks, uint32_t nkeys,
                                                                   const uint32_t* count, const uint32_t* offset,
                                                                   const uint32_t* chunk_off, const uint32_t* list,
                                                                   const G2AStore* S, G2JStore* out) {
  uint32_t c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= max_chunks || c >= chunk_off[nkeys]) return;
  uint32_t lo = 0, hi = nkeys;
  while (hi - lo > 1) {
    uint32_t mid = (lo + hi) / 2;
    if (chunk_off[mid] <= c)
      lo = mid;
    else
      hi = mid;
  }
  uint32_t first = offset[lo] + (c - chunk_off[lo]) * KMSM_CHUNK;
  uint32_t last = offset[lo] + count[lo];
  if (last > first + KMSM_CHUNK) last = first + KMSM_CHUNK;
#if DG_MSM_LDS
#if DG_MSM_LDS == 1
  __shared__ G2JStore s_acc[128];
  G2JStore& acc = s_acc[threadIdx.x];
#else
  G2JStore acc;
#endif
  store_g2j(acc, jac_from_aff(load_g2a(S[list[first]])));
  for (uint32_t i = first + 1; i < last; ++i) {
    const G2AStore& q = S[list[i]];
    if (!q.inf) g2_madd_lds(acc, q.x, q.y);  // the identity encoding decodes (status OK)
  }
  out[c] = acc;
#else
  G2J acc = jac_from_aff(load_g2a(S[list[first]]));
  for (uint32_t i = first + 1; i < last; ++i) {
    const G2AStore& q = S[list[i]];
    if (!q.inf) acc = g2_madd_lean(acc, q.x, q.y);  // the identity encoding decodes (status OK)
  }
  store_g2j(out[c], acc);
#endif
}
// lane = bucket key: sum of its chunks (identity when empty), the running sum in LDS (g2_add_lds)
DG_KERNEL void __launch_bounds__(128, DG_MSM_WAVES) k_kmsm_buckets(uint32_t nkeys, const uint32_t* chunk_off,
                                                                   const G2JStore* chunks, G2JStore* B) {
  uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= nkeys) return;
  __shared__ G2JStore s_acc[128];
  G2JStore& acc = s_acc[threadIdx.x];
  store_g2j(acc, jac_infinity<Fp2>());
  for (uint32_t c = chunk_off[b]; c < chunk_off[b + 1]; ++c) g2_add_lds(acc, load_g2j(chunks[c]));
  B[b] = acc;
}
// ---- Keyed MSM with affine first levels (msm_run_keyed): the entries of every (window, digit, set) bucket -- the
// decoded signatures, affine -- summed pairwise in MSM_AFF_L levels of affine additions with one batch inversion per
// level, as the single-key levels above (k_msm_aff_*), over the keyed list; then one lane per bucket adds its
// chunk sums A[offset[b] + c 2^L] with mixed additions.  About 15 Fp products per addition instead of the 29 of
// a mixed Jacobian addition in the chunk sums.  gofs: the level's group offsets per bucket (k_kscan_* with
// div = 2^(l+1)).
DG_KERNEL void __launch_bounds__(128) k_kmsm_aff_den(uint32_t l, uint32_t maxg, uint32_t nkeys, const uint32_t* count,
                                                     const uint32_t* offset, const uint32_t* gofs, const uint32_t* list,
                                                     const G2AStore* S, const G2AStore* A, Fp* den) {
  const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= maxg) return;
  Fp n = fp_one();
  uint32_t i, end;
  if (g < gofs[nkeys] && aff_group(nkeys, count, offset, gofs, l, g, i, end)) {
    const uint32_t j = i + (1u << l);
    const G2AStore &a = l == 0 ? S[list[i]] : A[i], &b = l == 0 ? S[list[j]] : A[j];
    if (!a.inf && !b.inf) {
      if (!fp2_eq(a.x, b.x))
        n = fp2_norm(fp2_sub(b.x, a.x));
      else if (fp2_eq(a.y, b.y))
        n = fp2_norm(fp2_dbl(a.y));
    }
  }
  den[g] = n;
}
DG_KERNEL void __launch_bounds__(128, DG_HOT_WAVES) k_kmsm_aff_add(uint32_t l, uint32_t maxg, uint32_t nkeys,
                                                                  const uint32_t* count, const uint32_t* offset,
                                                                  const uint32_t* gofs, const uint32_t* list,
                                                                  const G2AStore* S, G2AStore* A, const Fp* ninv) {
  const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= maxg || g >= gofs[nkeys]) return;
  uint32_t i, end;
  const bool pair = aff_group(nkeys, count, offset, gofs, l, g, i, end);
  if (!pair && l > 0) return;  // the lone entry already sits at i
  const G2A p = aff_srcA(l == 0 ? S[list[i]] : A[i]);
  if (!pair) {
    store_g2a(A[i], p);
    return;
  }
  const G2A q = aff_srcA(l == 0 ? S[list[i + 1]] : A[i + (1u << l)]);
  store_g2a(A[i], g2_aff_sum(p, q, g2_aff_kind(p, q), ninv[g]));
}
// lane (bucket key b, q < KMSM_BSPLIT): chunk sums q, q + KMSM_BSPLIT, ... of bucket b with mixed additions, the
// running sum in LDS, into BP[b * KMSM_BSPLIT + q] (then row-summed): ~400 points per bucket at C3 leave ~50 chunk
// sums, which one lane per bucket added in a long dependent chain
DG_KERNEL void __launch_bounds__(128, DG_MSM_WAVES) k_kmsm_buckets_aff(uint32_t nkeys, const uint32_t* count,
                                                                       const uint32_t* offset, const G2AStore* A,
                                                                       G2JStore* BP) {
  const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= nkeys * KMSM_BSPLIT) return;
  const uint32_t b = g / KMSM_BSPLIT, q = g % KMSM_BSPLIT;
  __shared__ G2JStore s_acc[128];
  G2JStore& acc = s_acc[threadIdx.x];
  store_g2j(acc, jac_infinity<Fp2>());
  const uint32_t nch = (count[b] + (1u << MSM_AFF_L) - 1) >> MSM_AFF_L;
  const G2AStore* Ab = A + offset[b];
  for (uint32_t c = q; c < nch; c += KMSM_BSPLIT) {
    const G2AStore& a = Ab[c << MSM_AFF_L];
    if (!a.inf) g2_madd_lds(acc, a.x, a.y);
  }
  BP[g] = acc;
}
#elif defined(__HIP__)
DG_KERNEL void __launch_bounds__(128) k_kmsm_aff_den(uint32_t l, uint32_t maxg, uint32_t nkeys, const uint32_t* count,
                                                     const uint32_t* offset, const uint32_t* gofs, const uint32_t* list,
                                                     const G2AStore* S, const G2AStore* A, Fp* den);
DG_KERNEL void __launch_bounds__(128, DG_HOT_WAVES) k_kmsm_aff_add(uint32_t l, uint32_t maxg, uint32_t nkeys,
                                                                  const uint32_t* count, const uint32_t* offset,
                                                                  const uint32_t* gofs, const uint32_t* list,
                                                                  const G2AStore* S, G2AStore* A, const Fp* ninv);
DG_KERNEL void __launch_bounds__(128, DG_MSM_WAVES) k_kmsm_buckets_aff(uint32_t nkeys, const uint32_t* count,
                                                                       const uint32_t* offset, const G2AStore* A,
                                                                       G2JStore* BP);
DG_KERNEL void __launch_bounds__(128, DG_MSM_WAVES) k_kmsm_buckets(uint32_t nkeys, const uint32_t* chunk_off,
                                                                   const G2JStore* chunks, G2JStore* B);
DG_KERNEL void __launch_bounds__(128, DG_MSM_WAVES) k_kmsm_chunks(uint32_t max_chunks, uint32_t nkeys,
                                                                   const uint32_t* count, const uint32_t* offset,
                                                                   const uint32_t* chunk_off, const uint32_t* list,
                                                                   const G2AStore* S, G2JStore* out);
#endif
#if defined(__HIP__) && DG_TU_LIB

// lane (set, w, k, c < 16): 8 of the buckets of (set, w) whose digit has bit k set; rows (set, w, k)
DG_KERNEL void __launch_bounds__(128, DG_BULK_WAVES) k_kmsm_slices(uint32_t nsets, uint32_t nwin, const G2JStore* B,
                                                                   G2JStore* P1) {
  uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= nsets * nwin * MSM_C * 16) return;
  uint32_t c = g % 16, k = (g / 16) % MSM_C, w = (g / (16 * MSM_C)) % nwin, set = g / (16 * MSM_C * nwin);
  G2J acc = jac_infinity<Fp2>();
  for (uint32_t i = 8 * c; i < 8 * c + 8; ++i) {
    uint32_t d = ((i >> k) << (k + 1)) | (1u << k) | (i & ((1u << k) - 1));
    acc = jac_add(acc, load_g2j(B[kmsm_key(w, d, set, nsets)]));
  }
  store_g2j(P1[g], acc);
}

// one 128-lane workgroup per set s: beta_s T_s by cooperative double-and-add (coop.h; beta is odd, so
// non-zero)
DG_KERNEL void __launch_bounds__(128, DG_COOP_WAVES) k_kmsm_beta(const uint64_t* seedp, const G2JStore* Tset, G2JStore* out) {
  DG_HI();
  const uint64_t seed = *seedp;
  __shared__ CoG2Tmp tmp;
  __shared__ CoG2 acc, p;
  const uint32_t s = blockIdx.x;
  const uint64_t beta = rlc_beta(seed, s);
  CO_SERIAL({
    G2J a = load_g2j(Tset[s]);
    p = CoG2{a.x, a.y, a.z};
    acc = p;
  });
  int top = 63;
  while (!((beta >> top) & 1)) --top;
  for (int b = top - 1; b >= 0; --b) {
    co_g2_dbl(&acc, &tmp);
    if ((beta >> b) & 1) co_g2_add(&acc, &acc, &p, &tmp);
  }
  CO_SERIAL(store_g2j(out[s], G2J{acc.x, acc.y, acc.z}));
}

#endif

}  // namespace dg
