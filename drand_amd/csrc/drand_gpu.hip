// libdrandgpu.so: the C-ABI of include/drand_gpu.h over the HIP kernels of kernels.h (gfx950 only).
// Host code here only moves bytes, sizes launches and sequences kernels; every group/field operation
// runs on the device.  No CPU fallback exists: without a gfx950 device the API returns DG_E_NODEV.
#include <chrono>
#include <hip/hip_runtime.h>

#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <functional>
#include <mutex>
#include <random>
#include <string>
#include <vector>

#include "../../include/drand_gpu.h"
#include "kernels.h"

using namespace dg;

namespace {

const uint8_t kDstNul[] = "BLS_SIG_BLS12381G2_XMD:SHA-256_SSWU_RO_NUL_";
constexpr uint32_t kDstNulLen = 43;

struct Timing {
  const char* name;
  double total_us;
  int launches;
};

// A workspace set: its own stream, grow-only device buffers and completion event.  Batches enqueued
// through the asynchronous entry point rotate over kSets sets, so the latency-bound tail of one batch
// (Miller loops, final exponentiation: a few workgroups) overlaps the throughput-bound head of the next.
#ifndef DG_MAX_SETS
#define DG_MAX_SETS 12
#endif
constexpr int kSets = DG_MAX_SETS;  // capacity; DG_SETS (environment) overrides the plan below
// The workspace plan for a hardware queue count (GPU_MAX_HW_QUEUES; HIP's default 4).  HIP binds streams to queues as
// they first dispatch (1, 2, 3, 4, 4, 3, 2, 1, 4, 3, ... on the box), a queue runs its streams' kernels one after
// another, and a cross-stream wait queued on a shared queue stalls every stream behind it:
//   >= 12 queues: 10 sets;  5..11 queues: queues - 2 sets (no two library streams share a queue, the caller keeps
//   one);  <= 4 queues: a multiple of the queue count (8 at 4), each queue carrying the same share of batches.
// The per-item passes (the check pipeline, checks.h / xr.h: every kernel under ~4 KB of private segment) run on the
// batch's own stream at every queue count (*per_item_on_set = 1); only the fixture kernels k_sign / k_hash_to_g2
// (~5.4 KB) keep a stream of their own, so no workspace queue reserves their scratch.
void queue_plan(int hwq, int* sets, int* per_item_on_set) {
  if (hwq < 1) hwq = 4;
  int v;
  if (hwq >= 12)
    v = 10;
  else if (hwq > 4)
    v = hwq - 2;
  else
    v = (10 / hwq) * hwq;
  v = v < 1 ? 1 : (v > kSets ? kSets : v);
  *sets = v;
  *per_item_on_set = 1;
}
int env_hw_queues() {
  const char* q = getenv("GPU_MAX_HW_QUEUES");
  return q && atoi(q) > 0 ? atoi(q) : 4;
}
int active_sets() {
  static const int n = [] {
    if (const char* e = getenv("DG_SETS")) {
      const int v = atoi(e);
      return v < 1 ? 1 : (v > kSets ? kSets : v);
    }
    int sets, shared;
    queue_plan(env_hw_queues(), &sets, &shared);
    return sets;
  }();
  return n;
}
// items per group test in Recover's per-item pass (kernels.h verify_group); DG_GROUP=1 or dg_set_group_size(1):
// every item alone
uint32_t g_group_size = [] {
  const char* e = getenv("DG_GROUP");
  int v = e ? atoi(e) : (int)GRP;
  return (uint32_t)(v < 1 ? 1 : (v > (int)GRP ? (int)GRP : v));
}();
uint32_t group_size() { return g_group_size; }
struct Set {
  hipStream_t stream = nullptr;
  std::vector<void*> pool;  // indexed by Slot
  std::vector<size_t> pool_size;
  hipEvent_t done = nullptr;
  bool busy = false;
  // the latency-bound end of this set's beacon batches (MSM row sums and Horner, the Miller loops and final
  // exponentiation of the batch equation, the cross-round isolation) runs on a high-priority stream: HIP gives those
  // hardware queues of their own beside the GPU_MAX_HW_QUEUES normal ones (tools/microbench/queue_prio.hip), so a
  // batch's few-workgroup tail no longer holds one of the 4 queues the bulk kernels share.  hop: the set stream's
  // bulk part done (the tail stream waits for it).
  hipStream_t tail = nullptr;
  int tail_idx = -1;  // which of Ctx::tails (and of Ctx::xr_pools: the sets sharing a tail stream share its pool)
  hipEvent_t hop = nullptr;
};

int env_int(const char* name, int dflt) {
  const char* e = getenv(name);
  return e ? atoi(e) : dflt;
}

struct Ctx {
  int device = -1;
  bool ready = false;
  Set sets[kSets];
  // the fixture kernels k_sign / k_hash_to_g2 (~5.4 KB of private segment per lane, the largest of the library) run
  // on this stream of their own: a hardware queue reserves scratch for the largest private segment dispatched on it,
  // for every wave the device can hold, so the workspace queues stay at the check pipeline's ~4 KB (12 workspace
  // queues at 5.7 KB each failed dg_init with HSA_STATUS_ERROR_OUT_OF_RESOURCES)
  hipStream_t fb_stream = nullptr;
  // the keyed batches' side stream (k_key_combine and Kc beside the keyed MSM; dg_init): the multi-key entry points
  // block until their batch is done, which the shared fork / join events rely on
  hipStream_t kc_stream = nullptr;
  hipEvent_t kc_fork = nullptr, kc_join = nullptr;
  static constexpr int kTails = 4;
  hipStream_t tails[kTails] = {};  // high-priority streams, by rotation position (Set::tail_idx; DG_TAIL=0: none)
  int ntails = 0;
  // the cross-round isolation's workspace (xr.h: ~0.8 GB at its capacity) per TAIL stream, not per set: the sets that
  // share a tail stream run their isolations one after another in that stream's order, so they can share its buffers
  // (4 copies instead of one per set).  xr_pool >= 0 while xr_isolate allocates (ws() takes that pool).
  Set xr_pools[kTails];
  int xr_pool = -1;
  hipStream_t last_stream = nullptr;  // the set stream of the last asynchronous batch (dg_last_batch_stream)
  int cur = 0, next = 0;
  bool timing = false;
  std::vector<Timing> timings;
  std::vector<std::pair<hipEvent_t, hipEvent_t>> pending;
  std::vector<const char*> pending_names;
  std::vector<hipEvent_t> free_events;
  // decoded group key of the single-key paths, shared by all sets (kyber keeps it decoded as well)
  G1AStore* pk_dev = nullptr;
  uint8_t* pk_status = nullptr;
  uint8_t* pk_raw = nullptr;
  hipEvent_t pk_ready = nullptr;
  uint8_t pk_bytes[48];
  bool pk_valid = false;
  unsigned long long* fallbacks = nullptr;  // device counter (k_count_fallback)
  unsigned long long* gcount = nullptr;     // device counters: group checks by member count (checks.h k_ck_prep)
  unsigned long long* xrcount = nullptr;    // device counters: cross-round isolation checks by level (xr.h)
  // share keys X_i = PubPoly.Eval(i) of the multi-key paths for the last (commits, distinct indices):
  // a drand group verifies every round against the same polynomial (the reference's build caches X_i
  // per group too), and decode + Horner are latency-bound single-lane jobs of ~15 ms
  G1AStore* poly_keys = nullptr;
  uint8_t* poly_kst = nullptr;
  size_t poly_cap = 0;
  hipEvent_t poly_ready = nullptr;
  std::vector<uint8_t> poly_commits;
  std::vector<uint32_t> poly_idx;
  bool poly_valid = false;
  // hash-to-G2 DST of sign / verify / recover (dg_set_hash_dst; default the NUL DST)
  std::vector<uint8_t> dst = std::vector<uint8_t>(kDstNul, kDstNul + kDstNulLen);
  // the DST and its word-wise expand_message_xmd tail, resident on the device (uploaded once per DST, never
  // inside a batch: a pageable host-to-device copy blocks the host until the stream reaches it, which would
  // serialise the asynchronous batches)
  XmdTail xmd;
  uint8_t* d_dst = nullptr;
  XmdTail* d_xmd = nullptr;
  bool dst_dev_valid = false;
  // single-key MSM bucket stage (msm_run): lanes per bucket over the affine chunk sums, and the row-sum fan-in of
  // their partials and of the slice partials (pairwise levels: each level is one dependent addition per lane, and
  // longer chains on a nearly empty chip measured slower)
  static constexpr uint32_t msm_bsplit = MSM_BSPLIT, msm_fold = 2, slice_fold = 2;
};

std::mutex g_mu;
Ctx g_ctx;

// HIP's hardware queues per process (GPU_MAX_HW_QUEUES, default 4) are read once, when the runtime starts (the
// process's first HIP call).  The library keeps up to 10 batches in flight on streams of their own, and with 4 queues
// those streams share queues: a cross-stream wait queued on a shared queue holds every stream behind it (DESIGN.md
// §5.3).  So when the library is loaded and the process has not chosen a value, it asks for kDefaultHwQueues -- for a
// program linked against it (the cgo drand binary) this runs before main, so before any HIP call.  An explicit
// GPU_MAX_HW_QUEUES (any value) is kept.  A process that started HIP BEFORE loading the library (torch imported and
// used first, with the variable unset) keeps HIP's 4 queues while the environment says 16: dg_init cannot query the
// runtime's count, so it warns once when the value is the library's own (g_hwq_supplied) -- such a process should set
// GPU_MAX_HW_QUEUES before its first HIP call (bench.py does).
constexpr const char* kDefaultHwQueues = "16";
bool g_hwq_supplied = false;
__attribute__((constructor)) void dg_default_hw_queues() {
  if (!getenv("GPU_MAX_HW_QUEUES")) {
    setenv("GPU_MAX_HW_QUEUES", kDefaultHwQueues, 0);
    g_hwq_supplied = true;
  }
}
thread_local std::string g_err;

int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

#define HIPCHK(expr)                                                                              \
  do {                                                                                            \
    hipError_t e_ = (expr);                                                                       \
    if (e_ != hipSuccess) return fail(DG_E_HIP, std::string(#expr) + ": " + hipGetErrorString(e_)); \
  } while (0)

// workspace slots
enum Slot {
  S_MSGS, S_DST, S_Q, S_S, S_U, S_STATUS, S_ISO, S_CELL, S_W, S_A, S_TMP, S_KP, S_F, S_H, S_FLAG, S_KEYS, S_KEYST, S_XC, S_FIN, S_LIST,
  S_COMMITS, S_COMMITST, S_SLOTIDX, S_ITEMSLOT, S_SEL, S_SELIDX, S_RST, S_SST, S_TERMS, S_IN0, S_IN1, S_IN2, S_IN3,
  S_IN4, S_OUT0, S_PK1, S_PK1ST, S_PK1RAW, S_ACTIVE, S_MSM_CNT, S_MSM_LIST, S_MSM_CHUNKS, S_MSM_B, S_MSM_G,
  S_MSM_P1, S_MSM_W, S_MSM_OUT, S_KMSM_CNT, S_KMSM_TOT, S_KMSM_LIST, S_KMSM_CHUNKS, S_KMSM_B, S_KMSM_P1,
  S_KMSM_TMP, S_KMSM_W, S_KMSM_T, S_KMSM_BT, S_DIG0, S_DIG1, S_SEED, S_VST, S_XMD, S_H2CST, S_EIN, S_EOUT, S_ISOPT, S_DECST, S_DEIN, S_DEOUT, S_BINV, S_NV, S_NVINV,
  S_IDXCNT, S_IDXFIRST, S_SLOTOF, S_MSM_AFF, S_MSM_DEN, S_MSM_DINV, S_BINV_PRE, S_BINV_ROOTS, S_RC_UNI, S_RC_REF, S_RC_LIST, S_RS_DIG,
  S_RC_NAF, S_RC_EV, S_RC_TAB, S_RC_D, S_RC_PINF, S_RC_DEN, S_RC_A, S_PW, S_SLOTW, S_SFULL, S_STFULL, S_INC, S_PB, S_SLOTB,
  S_SEED2, S_SB, S_STB, S_ISOB, S_KMSM_GOFS, S_KMSM_BP, S_KMSM_BT2,
  S_CK_RL, S_CK_HINF, S_CK_ST, S_CK_L2, S_CK_F, S_CK_T0, S_CK_T1, S_CK_F2, S_CK_A, S_CK_NV, S_CK_SN, S_CK_ZERO,
  S_CK_ZL, S_CK_GOOD, S_CK_T4, S_CK_TINF, S_CK_DIG, S_CK_TDEN, S_CK_BJ, S_CK_BN, S_CK_G2M, S_KOK, S_XR_CNT, S_XR_CAND,
  S_XR_QS, S_XR_T4, S_XR_TINF, S_XR_L3, S_XR_HS,
  // msm_run / batch_inv on the keyed batches' side stream (alt): the same buffers, apart from the main stream's
  S_MSM2_CNT, S_MSM2_LIST, S_MSM2_CHUNKS, S_MSM2_AFF, S_MSM2_DEN, S_MSM2_DINV, S_MSM2_B, S_MSM2_G, S_MSM2_P1, S_MSM2_W,
  S_MSM2_OUT, S_BINV2_PRE, S_BINV2_ROOTS, S_BINV2, S_COUNT
};

Set& cur_set() { return g_ctx.sets[g_ctx.cur]; }

// DG_HOSTPROF=1 (diagnostics): host time inside kernel launches and inside the set waits of acquire_set, printed and
// reset by dg_wait_all
struct HostProf {
  bool on = getenv("DG_HOSTPROF") != nullptr;
  double launch_us = 0, wait_us = 0;
  uint64_t launches = 0, waits = 0;
} g_hp;
// DG_BATCH_TRACE=1 (diagnostics): per asynchronous beacon batch, timing events at its start on the set stream, at
// the hand-over to its tail stream (hop) and at its end; printed (ms from the first start) and reset by dg_wait_all
struct BatchTrace {
  int set;
  hipEvent_t s, h, d;
};
struct BatchTraces {
  bool on = getenv("DG_BATCH_TRACE") != nullptr;
  std::vector<BatchTrace> v;
  BatchTrace* cur = nullptr;
} g_bt;
hipEvent_t bt_event(hipStream_t st) {
  hipEvent_t e = nullptr;
  if (hipEventCreate(&e) == hipSuccess) (void)hipEventRecord(e, st);
  return e;
}
inline double hp_now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int ws(Slot s, size_t bytes, void** out) {
  Set& c = g_ctx.xr_pool >= 0 ? g_ctx.xr_pools[g_ctx.xr_pool] : cur_set();
  if (c.pool.size() < S_COUNT) {
    c.pool.assign(S_COUNT, nullptr);
    c.pool_size.assign(S_COUNT, 0);
  }
  if (bytes == 0) bytes = 16;
  if (c.pool_size[s] < bytes) {
    // A slot grows while kernels enqueued earlier may still read it: this batch's own earlier launches (batch_inv
    // takes the same slots at several sizes), or, for a tail pool, another set's isolation.  The old buffer is freed
    // only after the device is idle, whatever hipFree itself waits for.  Slots only grow, so this happens in the first
    // batches of a size and never in the steady state.
    if (c.pool[s]) {
      HIPCHK(hipDeviceSynchronize());
      HIPCHK(hipFree(c.pool[s]));
    }
    c.pool[s] = nullptr;
    size_t sz = bytes + bytes / 4;
    HIPCHK(hipMalloc(&c.pool[s], sz));
    c.pool_size[s] = sz;
  }
  *out = c.pool[s];
  return 0;
}

// The order in which batches take the workspace sets.  HIP binds the set streams to its hardware queues as they first
// dispatch (dg_init's prewarm, sets 0, 1, 2, ...), and at 4 queues the binding zigzags: sets 0..7 on queues 1, 2, 3, 4,
// 4, 3, 2, 1.  Taking the sets in index order sent batches 3, 4 to queue 4 and 7, 0 to queue 1, so a
// window of 20 batches gave queue 4 six heads and queue 1 four, and the region waited for queue 4 alone at its end
// (DESIGN.md §5.5).  With 8 sets on 4 queues the order 0, 1, 2, 3, 7, 6, 5, 4 visits queues 1, 2, 3, 4, 1, 2, 3, 4:
// every window of batches is spread over the queues to within one.
int set_at(int slot) {
  const int n = active_sets();
  if (n != 8 || env_hw_queues() != 4) return slot;
  static const int order[8] = {0, 1, 2, 3, 7, 6, 5, 4};
  return order[slot];
}
// Take the next workspace set (waiting for the batch still using it) and make it current.
int acquire_set(hipStream_t* st) {
  Ctx& c = g_ctx;
  const int i = set_at(c.next);
  c.next = (c.next + 1) % active_sets();
  Set& s = c.sets[i];
  if (s.busy) {
    const double h0 = g_hp.on ? hp_now_us() : 0.0;
    HIPCHK(hipEventSynchronize(s.done));
    if (g_hp.on) {
      g_hp.wait_us += hp_now_us() - h0;
      ++g_hp.waits;
    }
    s.busy = false;
  }
  c.cur = i;
  *st = s.stream;
  return 0;
}

// The multi-key blocking entry points (VerifyPartial, Recover) always take set 0 (waiting for a batch still using
// it): their grow-only buffers are the largest (~20 GB at 100k rounds x 64 partials: the keyed MSM's affine entry
// array), and rotating them over every set would hold one such copy per set.
int acquire_set0(hipStream_t* st) {
  Ctx& c = g_ctx;
  Set& s = c.sets[0];
  if (s.busy) {
    HIPCHK(hipEventSynchronize(s.done));
    s.busy = false;
  }
  c.cur = 0;
  *st = s.stream;
  return 0;
}

hipEvent_t get_event() {
  Ctx& c = g_ctx;
  if (!c.free_events.empty()) {
    hipEvent_t e = c.free_events.back();
    c.free_events.pop_back();
    return e;
  }
  hipEvent_t e;
  (void)hipEventCreate(&e);
  return e;
}

// launch helper with optional per-kernel event timing
template <typename... Args>
int launch_shm(const char* name, void (*k)(Args...), uint32_t n_threads, uint32_t block, uint32_t shm, hipStream_t st,
               Args... args);
template <typename... Args>
int launch(const char* name, void (*k)(Args...), uint32_t n_threads, uint32_t block, hipStream_t st, Args... args) {
  return launch_shm(name, k, n_threads, block, 0u, st, args...);
}
template <typename... Args>
int launch_shm(const char* name, void (*k)(Args...), uint32_t n_threads, uint32_t block, uint32_t shm, hipStream_t st,
               Args... args) {
  if (n_threads == 0) return 0;
  const uint32_t grid = (uint32_t)(((uint64_t)n_threads + block - 1) / block);
  Ctx& c = g_ctx;
  hipEvent_t e0 = nullptr, e1 = nullptr;
  if (c.timing) {
    e0 = get_event();
    e1 = get_event();
    (void)hipEventRecord(e0, st);
  }
  const double h0 = g_hp.on ? hp_now_us() : 0.0;
  hipLaunchKernelGGL(k, dim3(grid), dim3(block), shm, st, args...);
  if (g_hp.on) {
    g_hp.launch_us += hp_now_us() - h0;
    ++g_hp.launches;
  }
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return fail(DG_E_HIP, std::string("launch ") + name + ": " + hipGetErrorString(e));
  if (c.timing) {
    (void)hipEventRecord(e1, st);
    c.pending.push_back({e0, e1});
    c.pending_names.push_back(name);
  }
  return 0;
}

void collect_timings() {
  Ctx& c = g_ctx;
  for (size_t i = 0; i < c.pending.size(); ++i) {
    float ms = 0;
    (void)hipEventSynchronize(c.pending[i].second);
    (void)hipEventElapsedTime(&ms, c.pending[i].first, c.pending[i].second);
    bool found = false;
    for (auto& t : c.timings)
      if (t.name == c.pending_names[i]) {
        t.total_us += ms * 1e3;
        t.launches++;
        found = true;
      }
    if (!found) c.timings.push_back({c.pending_names[i], ms * 1e3, 1});
    c.free_events.push_back(c.pending[i].first);
    c.free_events.push_back(c.pending[i].second);
  }
  c.pending.clear();
  c.pending_names.clear();
}

int require_ready() {
  if (!g_ctx.ready) return fail(DG_E_NODEV, "dg_init() has not selected a gfx950 device");
  return 0;
}

uint64_t fresh_seed(uint64_t seed) {
  if (seed) return seed;
  std::random_device rd;
  return ((uint64_t)rd() << 32) ^ rd() ^ 0x9e3779b97f4a7c15ull;
}

#define RET(expr)          \
  do {                     \
    int r_ = (expr);       \
    if (r_ != 0) return r_; \
  } while (0)

template <typename T>
int upload(Slot s, const T* host, size_t count, T** dev, hipStream_t st) {
  void* p;
  RET(ws(s, sizeof(T) * count, &p));
  if (count) HIPCHK(hipMemcpyAsync(p, host, sizeof(T) * count, hipMemcpyHostToDevice, st));
  *dev = (T*)p;
  return 0;
}

template <typename T>
int wsT(Slot s, size_t count, T** out) {
  void* p;
  RET(ws(s, sizeof(T) * count, &p));
  *out = (T*)p;
  return 0;
}

// Collapse each of `rows` rows of `cols` Jacobian points (row-major in buf) to its sum, left in buf[row].
// Pairwise levels by default (one dependent addition per lane per launch): these launches run on a nearly
// empty chip, so their time is the depth of the addition chain, not the number of additions.
// skip (device, may be null): rows of a block of 64 with skip[row / 64] != 0 are not summed (their result is garbage).
int reduce_rows(G2JStore* buf, G2JStore* tmp, uint32_t rows, uint32_t cols, hipStream_t st, uint32_t max_chunk = 2,
                const uint8_t* skip = nullptr) {
  G2JStore* src = buf;
  G2JStore* dst = tmp;
  while (cols > 1) {
    uint32_t chunk = cols < max_chunk ? cols : max_chunk;
    uint32_t ocols = (cols + chunk - 1) / chunk;
    RET(launch("k_sum_rows", k_sum_rows, rows * ocols, 128, st, rows, cols, chunk, (const G2JStore*)src, dst, skip));
    cols = ocols;
    std::swap(src, dst);
  }
  if (src != buf) HIPCHK(hipMemcpyAsync(buf, src, sizeof(G2JStore) * rows, hipMemcpyDeviceToDevice, st));
  return 0;
}

// One batch of the verification engine (kernels.h): R rounds with uncleared hashes Q, k items per round,
// nslots keys.  Fills S / status / isolate for the N = R*k items; status ends as the exact per-item
// bls.Verify verdict.
struct Batch {
  uint32_t R, k, nslots;      // nslots: key slots in the batch equation; items of slots >= nslots are checked alone
  const G2JStore* Q;
  const G1AStore* keys;       // every item's key (slots >= nslots included)
  const uint8_t* key_status;
  const uint32_t* item_slot;  // N entries, or null when nslots == 1
  const uint8_t* sigs;        // N records of `stride` bytes, sigma at `offset`
  uint32_t stride, offset;
  G2AStore* S;
  uint8_t* status;
  const uint8_t* msgs;        // R messages of msg_len bytes (device): bound into the batch coefficients
  uint32_t msg_len;
  const uint8_t* key_bytes;   // host: the key encoding(s) (48 B pk, or t x 48 B commits)
  size_t key_len;
  bool item_pass = true;  // false (Recover's window): stop after the batch equation, verdicts in BatchOut
};
// what a batch without its per-item pass leaves for the caller (device pointers, valid in stream order)
struct BatchOut {
  const uint64_t* seed = nullptr;  // the bound coefficient seed
  const uint32_t* flag = nullptr;  // flag[0]: the batch equation held
  const uint8_t* iso = nullptr;    // N: items the equation did not cover (isolated)
  uint32_t batched_sub = 0;        // 1: the G2 subgroup checks were batched (decode skipped them)
};

// The batch's coefficient seed (kernels.h k_digest_*): seed' = SHA-256(SHA-256(BE64 seed || key bytes) || D),
// D = a SHA-256 tree over every (message, signature record) of the batch, left on the device.
int bind_seed(const Batch& b, uint64_t seed, hipStream_t st, uint64_t** d_seed, Slot seed_slot = S_SEED) {
  const uint32_t N = b.R * b.k;
  Sha256 h;
  sha256_init(h);
  for (int i = 7; i >= 0; --i) sha256_byte(h, (uint8_t)(seed >> (8 * i)));
  sha256_update(h, b.key_bytes, (uint32_t)b.key_len);
  uint8_t seed0[32];
  sha256_final(h, seed0);
  // seed0 travels as a kernel argument: a host-to-device copy here would block the host (see ensure_dst)
  Seed0 s0;
  for (int i = 0; i < 8; ++i)
    s0.w[i] = (uint32_t)seed0[4 * i] << 24 | (uint32_t)seed0[4 * i + 1] << 16 | (uint32_t)seed0[4 * i + 2] << 8 | seed0[4 * i + 3];
  uint8_t *d0, *d1;
  RET(wsT(S_DIG0, (size_t)32 * N, &d0));
  RET(wsT(S_DIG1, (size_t)32 * ((N + 63) / 64) + 64, &d1));
  RET(wsT(seed_slot, 16, d_seed));
  RET(launch("k_digest_items", k_digest_items, N, 128, st, N, b.k, b.msgs, b.msg_len, b.sigs, b.stride, d0));
  uint32_t n = N;
  while (n > 1) {
    uint32_t m = (n + 63) / 64;
    RET(launch("k_digest_level", k_digest_level, m, 128, st, n, (const uint8_t*)d0, d1));
    std::swap(d0, d1);
    n = m;
  }
  return launch("k_digest_seed", k_digest_seed, 1, 64, st, s0, (const uint8_t*)d0, *d_seed);
}

// Pippenger MSM (msm.h): out[0] = sum_r alpha_r PA_r, out[1] = sum_r alpha_r PB_r (PB may be null),
// over the rounds with active[r] != 0.  With `test_windows` side A also gets the MSM_TWIN test windows of
// the batched subgroup check; *win = its MSM_WT window sums (checked beside the Miller loops, k_pair_miller_coop).
int batch_inv(uint32_t n, const Fp* vals, Fp* out, hipStream_t st, bool alt = false);

// the per-item passes after a batch equation (defined with the check pipeline below)
constexpr uint32_t kXrSeg = 131072;  // items per cross-round isolation run at most (bounded per-check workspace)
int xr_isolate(uint32_t i0, uint32_t n, const uint32_t* flag, const uint64_t* seed, const G1AStore* keys,
               const G2JStore* Q, const G2AStore* S, uint8_t* status, hipStream_t st);
int prefix_pass(uint32_t R, uint32_t k, uint32_t t, int passes, const uint64_t* seed, const G1AStore* keys,
                const uint32_t* item_slot, const G2JStore* Q, const G2AStore* S, uint8_t* status, uint8_t* fin,
                uint32_t subgroup, hipStream_t st);

// `affine`: every point of PA and PB has Z = 1 or Z = 0, so the first levels are affine additions (msm.h).
// `bad` (device, affine only): raised when an input breaks that precondition (msm.h aff_input_ok); the caller
// passes its batch-failure flag, so such a batch falls back to exact per-item checks.
int msm_run(uint32_t R, const uint64_t* seed, const uint8_t* active, const G2JStore* PA, const G2JStore* PB, bool test_windows,
            bool affine, G2JStore** out, G2JStore** win, hipStream_t st, uint32_t* bad = nullptr, hipStream_t tst = nullptr,
            bool alt = false) {
  const uint32_t nsides = PB ? 2 : 1, nwin = test_windows ? MSM_WT : MSM_WIN, nbk = nwin * MSM_NB;
  // alt: the side stream's copies of every buffer (it runs beside the keyed MSM, batch_verify)
  auto SL = [alt](Slot a, Slot b) { return alt ? b : a; };
  uint32_t *cnt, *list;
  G2JStore *chunks, *BP, *tmp, *P1, *W;
  RET(wsT(SL(S_MSM_CNT, S_MSM2_CNT), 4 * nbk + 1 + MSM_AFF_L * (nbk + 1), &cnt));
  uint32_t *offset = cnt + nbk, *cursor = offset + nbk, *chunk_off = cursor + nbk;
  RET(wsT(SL(S_MSM_LIST, S_MSM2_LIST), (size_t)nwin * R + 1, &list));
  if (affine && !bad) return fail(DG_E_ARG, "msm_run: the affine levels need a failure flag");
  if (affine) {
    const size_t E = (size_t)nwin * R;
    if (E * nsides > 0x7fffffffull) return fail(DG_E_ARG, "batch too large for the MSM");
    uint32_t* gofs = chunk_off + nbk + 1;
    G2AStore* A;
    Fp *den, *dinv;
    const uint32_t maxg0 = (uint32_t)(E / 2) + nbk;
    RET(wsT(SL(S_MSM_AFF, S_MSM2_AFF), E * nsides, &A));
    RET(wsT(SL(S_MSM_DEN, S_MSM2_DEN), (size_t)maxg0 * nsides, &den));
    RET(wsT(SL(S_MSM_DINV, S_MSM2_DINV), (size_t)maxg0 * nsides, &dinv));
    RET(wsT(SL(S_MSM_B, S_MSM2_B), (size_t)nbk * MSM_BSPLIT * nsides, &BP));
    RET(wsT(SL(S_MSM_G, S_MSM2_G), (size_t)nbk * MSM_BSPLIT * nsides, &tmp));
    RET(wsT(SL(S_MSM_P1, S_MSM2_P1), (size_t)nwin * MSM_C * MSM_SLICE_LANES * nsides, &P1));
    RET(wsT(SL(S_MSM_W, S_MSM2_W), (size_t)nwin * nsides, &W));
    RET(wsT(SL(S_MSM_OUT, S_MSM2_OUT), 2, out));
    HIPCHK(hipMemsetAsync(cnt, 0, sizeof(uint32_t) * nbk, st));
    RET(launch("k_msm_count", k_msm_count, R, 256, st, R, nwin, seed, active, cnt));
    RET(launch("k_msm_scan_aff", k_msm_scan_aff, 256, 256, st, nbk, (const uint32_t*)cnt, offset, cursor, gofs));
    RET(launch("k_msm_scatter", k_msm_scatter, R, 256, st, R, nwin, seed, active, cursor, list));
    for (uint32_t l = 0; l < MSM_AFF_L; ++l) {
      const uint32_t maxg = (uint32_t)(E >> (l + 1)) + nbk, n = maxg * nsides;
      const uint32_t* gl = gofs + l * (nbk + 1);
      RET(launch("k_msm_aff_den", k_msm_aff_den, n, 128, st, l, maxg, nsides, nbk, (const uint32_t*)cnt,
                 (const uint32_t*)offset, gl, (const uint32_t*)list, PA, PB, (const G2AStore*)A, (uint32_t)E, den));
      RET(batch_inv(n, den, dinv, st, alt));
      RET(launch("k_msm_aff_add", k_msm_aff_add, n, 128, st, l, maxg, nsides, nbk, (const uint32_t*)cnt,
                 (const uint32_t*)offset, gl, (const uint32_t*)list, PA, PB, A, (uint32_t)E, (const Fp*)dinv, bad));
    }
    RET(launch("k_msm_buckets_aff", k_msm_buckets_aff, nbk * g_ctx.msm_bsplit * nsides, 128, st, nsides, nbk,
               g_ctx.msm_bsplit, (const uint32_t*)cnt, (const uint32_t*)offset, (const G2AStore*)A, (uint32_t)E, BP));
    RET(reduce_rows(BP, tmp, nbk * nsides, g_ctx.msm_bsplit, st, g_ctx.msm_fold));  // B[side][b] = BP[side * nbk + b]
  } else {
  const size_t max_chunks_sz = ((size_t)nwin * R) / MSM_CHUNK + nbk;
  if (max_chunks_sz * nsides > 0xffffffffull) return fail(DG_E_ARG, "batch too large for the MSM");
  const uint32_t max_chunks = (uint32_t)max_chunks_sz;
  RET(wsT(SL(S_MSM_CHUNKS, S_MSM2_CHUNKS), (size_t)max_chunks * nsides, &chunks));
  RET(wsT(SL(S_MSM_B, S_MSM2_B), (size_t)nbk * MSM_BSPLIT * nsides, &BP));
  RET(wsT(SL(S_MSM_G, S_MSM2_G), (size_t)nbk * MSM_BSPLIT * nsides, &tmp));
  RET(wsT(SL(S_MSM_P1, S_MSM2_P1), (size_t)nwin * MSM_C * MSM_SLICE_LANES * nsides, &P1));
  RET(wsT(SL(S_MSM_W, S_MSM2_W), (size_t)nwin * nsides, &W));
  RET(wsT(SL(S_MSM_OUT, S_MSM2_OUT), 2, out));
  HIPCHK(hipMemsetAsync(cnt, 0, sizeof(uint32_t) * nbk, st));
  RET(launch("k_msm_count", k_msm_count, R, 256, st, R, nwin, seed, active, cnt));
  RET(launch("k_msm_scan", k_msm_scan, 256, 256, st, nbk, (const uint32_t*)cnt, offset, cursor, chunk_off));
  RET(launch("k_msm_scatter", k_msm_scatter, R, 256, st, R, nwin, seed, active, cursor, list));
  RET(launch("k_msm_chunks", k_msm_chunks, max_chunks * nsides, 128, st, max_chunks, nsides, nbk, (const uint32_t*)cnt,
             (const uint32_t*)offset, (const uint32_t*)chunk_off, (const uint32_t*)list, PA, PB, chunks));
  RET(launch("k_msm_buckets", k_msm_buckets, nbk * MSM_BSPLIT * nsides, 128, st, max_chunks, nsides, nbk,
             (const uint32_t*)chunk_off, (const G2JStore*)chunks, BP));
  RET(reduce_rows(BP, tmp, nbk * nsides, MSM_BSPLIT, st));  // B[side][b] = BP[side * nbk + b]
  }
  RET(launch("k_msm_slices", k_msm_slices, nsides * nwin * MSM_C * MSM_SLICE_LANES, 128, st, nsides, nwin, (const G2JStore*)BP, P1));
  if (tst) {
    // the rest is latency-bound: it moves to the batch's tail stream (Set::tail)
    HIPCHK(hipEventRecord(cur_set().hop, st));
    if (g_bt.cur) g_bt.cur->h = bt_event(st);
    HIPCHK(hipStreamWaitEvent(tst, cur_set().hop, 0));
    st = tst;
  }
  RET(reduce_rows(P1, tmp, nsides * nwin * MSM_C, MSM_SLICE_LANES, st, g_ctx.slice_fold));  // S[side][w][k] = P1[...]
  RET(launch("k_msm_horner_coop", k_msm_horner_coop, 128 * nwin * nsides, 128, st, nwin, 1u, (const G2JStore*)P1, W));
  RET(launch("k_msm_final_coop", k_msm_final_coop, 128 * nsides, 128, st, nwin, (const G2JStore*)W, *out));
  if (win) *win = W;
  return 0;
}

// Keyed MSM (msm.h) of the multi-key batch: T = sum_s beta_s sum_{items i of slot s} alpha_{r(i)} S_i.
// With `test_windows` every key set also gets the MSM_TWIN test windows; *win = the nsets x MSM_WT window
// sums of the batched subgroup check.
int msm_run_keyed(const Batch& b, const uint64_t* seed, const uint8_t* iso, bool test_windows, G2JStore** T, G2JStore** win,
                  hipStream_t st) {
  const uint32_t nwin = test_windows ? MSM_WT : MSM_WIN;
  const uint32_t N = b.R * b.k, nsets = b.nslots;
  if ((size_t)nwin * MSM_NB * nsets > 0x7fffffffull) return fail(DG_E_ARG, "too many key sets");
  const uint32_t nkeys = nwin * MSM_NB * nsets;
  const uint32_t nblocks = (nkeys + KSCAN_B - 1) / KSCAN_B;
  uint32_t *cnt, *tot, *list;
  G2JStore *chunks, *B, *P1, *tmp, *W, *Ts, *BT;
  RET(wsT(S_KMSM_CNT, (size_t)4 * nkeys + 1, &cnt));
  uint32_t *offset = cnt + nkeys, *cursor = offset + nkeys, *chunk_off = cursor + nkeys;  // chunk_off: nkeys + 1
  RET(wsT(S_KMSM_TOT, (size_t)2 * nblocks, &tot));
  RET(wsT(S_KMSM_LIST, (size_t)nwin * N + 1, &list));
  // sum of ceil(count / KMSM_CHUNK) <= nwin N / KMSM_CHUNK + nkeys
  const size_t max_chunks_sz = ((size_t)nwin * N) / KMSM_CHUNK + 1 + nkeys;
  if (max_chunks_sz > 0xffffffffull) return fail(DG_E_ARG, "batch too large for the keyed MSM");
  const uint32_t max_chunks = (uint32_t)max_chunks_sz;
  RET(wsT(S_KMSM_B, nkeys, &B));
  RET(wsT(S_KMSM_P1, (size_t)nsets * nwin * MSM_C * 16, &P1));
  RET(wsT(S_KMSM_TMP, (size_t)nsets * nwin * MSM_C * 16, &tmp));
  RET(wsT(S_KMSM_W, (size_t)nsets * nwin, &W));
  RET(wsT(S_KMSM_T, nsets, &Ts));
  RET(wsT(S_KMSM_BT, nsets, &BT));
  HIPCHK(hipMemsetAsync(cnt, 0, sizeof(uint32_t) * nkeys, st));
  RET(launch("k_kmsm_count", k_kmsm_count, N, 256, st, N, b.k, nsets, nwin, seed, b.item_slot, (const uint8_t*)b.status,
             iso, cnt));
  const size_t E = (size_t)nwin * N;
  const bool aff = E + nkeys < 0x7fffffffull;  // affine first levels (else: Jacobian chunk sums)
  auto scan = [&](uint32_t div, uint32_t* groups) -> int {
    RET(launch("k_kscan_local", k_kscan_local, nblocks * 256, 256, st, nkeys, div, (const uint32_t*)cnt, offset, groups,
               tot));
    RET(launch("k_kscan_top", k_kscan_top, 64, 64, st, nblocks, nkeys, tot, groups));
    return launch("k_kscan_add", k_kscan_add, nkeys, 256, st, nkeys, (const uint32_t*)tot, offset, cursor, groups);
  };
  uint32_t* gofs = nullptr;
  if (aff) {
    RET(wsT(S_KMSM_GOFS, (size_t)MSM_AFF_L * (nkeys + 1), &gofs));
    for (uint32_t l = 0; l < MSM_AFF_L; ++l) RET(scan(2u << l, gofs + (size_t)l * (nkeys + 1)));
  } else {
    RET(scan(KMSM_CHUNK, chunk_off));
  }
  RET(launch("k_kmsm_scatter", k_kmsm_scatter, N, 256, st, N, b.k, nsets, nwin, seed, b.item_slot,
             (const uint8_t*)b.status, iso, cursor, list));
  if (aff) {
    G2AStore* A;
    Fp *den, *dinv;
    const uint32_t maxg0 = (uint32_t)(E / 2) + nkeys;
    RET(wsT(S_MSM_AFF, E, &A));
    RET(wsT(S_MSM_DEN, maxg0, &den));
    RET(wsT(S_MSM_DINV, maxg0, &dinv));
    for (uint32_t l = 0; l < MSM_AFF_L; ++l) {
      const uint32_t maxg = (uint32_t)(E >> (l + 1)) + nkeys;
      const uint32_t* gl = gofs + (size_t)l * (nkeys + 1);
      RET(launch("k_kmsm_aff_den", k_kmsm_aff_den, maxg, 128, st, l, maxg, nkeys, (const uint32_t*)cnt,
                 (const uint32_t*)offset, gl, (const uint32_t*)list, (const G2AStore*)b.S, (const G2AStore*)A, den));
      RET(batch_inv(maxg, den, dinv, st));
      RET(launch("k_kmsm_aff_add", k_kmsm_aff_add, maxg, 128, st, l, maxg, nkeys, (const uint32_t*)cnt,
                 (const uint32_t*)offset, gl, (const uint32_t*)list, (const G2AStore*)b.S, A, (const Fp*)dinv));
    }
    G2JStore *BP, *BT2;
    RET(wsT(S_KMSM_BP, (size_t)nkeys * KMSM_BSPLIT, &BP));
    RET(wsT(S_KMSM_BT2, (size_t)nkeys * KMSM_BSPLIT, &BT2));
    RET(launch("k_kmsm_buckets_aff", k_kmsm_buckets_aff, nkeys * KMSM_BSPLIT, 128, st, nkeys, (const uint32_t*)cnt,
               (const uint32_t*)offset, (const G2AStore*)A, BP));
    RET(reduce_rows(BP, BT2, nkeys, KMSM_BSPLIT, st));  // BP[b] = bucket b
    B = BP;
  } else {
    RET(wsT(S_KMSM_CHUNKS, max_chunks, &chunks));
    RET(launch("k_kmsm_chunks", k_kmsm_chunks, max_chunks, 128, st, max_chunks, nkeys, (const uint32_t*)cnt,
               (const uint32_t*)offset, (const uint32_t*)chunk_off, (const uint32_t*)list, (const G2AStore*)b.S,
               chunks));
    RET(launch("k_kmsm_buckets", k_kmsm_buckets, nkeys, 128, st, nkeys, (const uint32_t*)chunk_off,
               (const G2JStore*)chunks, B));
  }
  RET(launch("k_kmsm_slices", k_kmsm_slices, nsets * nwin * MSM_C * 16, 128, st, nsets, nwin, (const G2JStore*)B, P1));
  RET(reduce_rows(P1, tmp, nsets * nwin * MSM_C, 16, st));  // S[set][w][k] = P1[...]
  RET(launch("k_msm_horner_coop", k_msm_horner_coop, 128 * nwin * nsets, 128, st, nwin, nsets, (const G2JStore*)P1, W));
  RET(launch("k_msm_final_coop", k_msm_final_coop, 128 * nsets, 128, st, nwin, (const G2JStore*)W, Ts));
  if (win) *win = W;
  RET(launch("k_kmsm_beta", k_kmsm_beta, 128 * nsets, 128, st, seed, (const G2JStore*)Ts, BT));
  RET(reduce_rows(BT, tmp, 1, nsets, st));  // T = BT[0]
  *T = BT;
  return 0;
}

// sigma decode of n items (96 B at sigs + stride * i + offset) into S / status; the (round, slot) cell claim of
// kernels.h (nslots = 0: no cell, every decoded item isolated); `sub`: the G2 subgroup check per item
int decode_items(uint32_t N, uint32_t k, uint32_t nslots, const uint8_t* sigs, uint32_t stride, uint32_t offset,
                 const uint32_t* item_slot, const uint8_t* key_status, G2AStore* S, uint8_t* status, uint32_t* cell,
                 uint8_t* iso, uint32_t sub, hipStream_t st) {
  // phases.h: flags / x, the two roots through k_exp_pm3d4, then y, sign and the cell claim
  DecState* ds;
  Fp *ein, *eout;
  RET(wsT(S_DECST, N, &ds));
  RET(wsT(S_DEIN, N, &ein));
  RET(wsT(S_DEOUT, N, &eout));
  RET(launch("k_dec_p1", k_dec_p1, N, 128, st, N, sigs, stride, offset, item_slot, key_status, ds, ein, status));
  RET(launch("k_exp_pm3d4", k_exp_pm3d4, N, 128, st, N, (const Fp*)ein, eout));
  RET(launch("k_dec_p2", k_dec_p2, N, 128, st, N, ds, ein, (const Fp*)eout, status));
  RET(launch("k_exp_pm3d4", k_exp_pm3d4, N, 128, st, N, (const Fp*)ein, eout));
  return launch("k_dec_p3", k_dec_p3, N, 128, st, N, k, nslots, item_slot, (const DecState*)ds, (const Fp*)ein,
                (const Fp*)eout, S, status, cell, iso, sub);
}

// tst (single key only, may be null): the stream the batch's latency-bound end runs on (Set::tail); the batch is
// complete in tst's order then
int batch_verify(const Batch& b, uint64_t seed_in, hipStream_t st, BatchOut* out = nullptr, hipStream_t tst = nullptr) {
  const uint32_t N = b.R * b.k;
  uint64_t* d_seed;
  RET(bind_seed(b, seed_in, st, &d_seed));
  const uint64_t* seed = d_seed;
  uint8_t *iso, *active;
  uint32_t *cell, *flag;
  G2JStore *U, *V, *A = nullptr, *tmp, *Kp, *msm;
  Fp12* f;
  RET(wsT(S_ISO, N, &iso));
  RET(wsT(S_ACTIVE, b.R, &active));
  RET(wsT(S_CELL, (size_t)b.R * b.nslots, &cell));
  RET(wsT(S_FLAG, 4, &flag));
  U = V = nullptr;
  if (b.nslots == 1) {
    RET(wsT(S_U, N, &U));
    RET(wsT(S_W, b.R, &V));
  } else {
    RET(wsT(S_A, b.R, &A));
  }
  RET(wsT(S_F, b.nslots + 2, &f));
  HIPCHK(hipMemsetAsync(cell, 0, sizeof(uint32_t) * (size_t)b.R * b.nslots, st));
  // one item per (round, key): the G2 subgroup checks of the signatures are batched on the MSM's window
  // sums (msm.h) instead of a psi check per item (several items of one key in a round share their digits)
  const uint32_t batched_sub = (b.nslots > 1 || b.k == 1) ? 1u : 0u;
  // flag[2]: the batch's failure flag beside the equation -- the batched subgroup check's window sums
  // (k_pair_miller_coop) and the affine MSM levels' input check (msm.h aff_input_ok) raise it
  HIPCHK(hipMemsetAsync(flag + 2, 0, 4, st));
  RET(decode_items(N, b.k, b.nslots, b.sigs, b.stride, b.offset, b.item_slot, b.key_status, b.S, b.status, cell, iso,
                   1u - batched_sub, st));
  if (b.nslots == 1)
    RET(launch("k_scale_items", k_scale_items, N, 128, st, N, b.nslots, seed, b.item_slot, (const G2AStore*)b.S,
               (const uint8_t*)b.status, (const uint8_t*)iso, U));
  RET(launch("k_round_combine", k_round_combine, b.R, 128, st, b.R, b.k, b.nslots, seed, (const G2JStore*)U,
             (const uint8_t*)b.status, (const uint8_t*)iso, b.Q, (const uint32_t*)cell, V, A, active));
  const G2JStore *T, *K, *Kc = nullptr;
  G1AStore* Xc = nullptr;
  G2JStore* win = nullptr;
  if (b.nslots == 1) {
    // T = sum alpha_r V_r and K = sum alpha_r Q_r in one MSM (shared bucket sort)
    RET(msm_run(b.R, seed, active, V, b.Q, batched_sub != 0, b.k == 1, &msm, &win, st, flag + 2, tst));
    if (tst) st = tst;
    T = msm;
    K = msm + 1;
  } else {
    // Xc = sum_s beta_s X_s (k_key_combine: one workgroup, ~2 ms of dependent doublings) and Kc on the side stream,
    // joined before the Miller launch: they need only the bound seed, the keys, the hashes and `active`, so they run
    // beside the keyed MSM below
    RET(wsT(S_XC, 1, &Xc));
    Ctx& c = g_ctx;
    // kc_fork / kc_join are global while the S_MSM2_* / S_BINV2_* buffers belong to the set: safe only because every
    // multi-key entry point blocks until its batch is done (one keyed batch in flight at a time)
    HIPCHK(hipEventRecord(c.kc_fork, st));
    HIPCHK(hipStreamWaitEvent(c.kc_stream, c.kc_fork, 0));
    RET(launch("k_key_combine", k_key_combine, 256, 256, c.kc_stream, b.nslots, seed, b.keys, b.key_status, Xc));
    // Kc = sum over the active rounds of alpha_r Q_r (one MSM, a ~3.4 ms chain of small launches at 100k rounds): on
    // the side stream too, in its own buffers
    G2JStore* kmsm;
    RET(msm_run(b.R, seed, active, b.Q, nullptr, false, true, &kmsm, nullptr, c.kc_stream, flag + 2, nullptr, true));
    Kc = kmsm;
    HIPCHK(hipEventRecord(c.kc_join, c.kc_stream));
    // T = sum_s beta_s sum_{i in s} alpha_{r(i)} S_i by the keyed MSM (no per-item scalar multiplication)
    RET(msm_run_keyed(b, seed, iso, batched_sub != 0, &msm, &win, st));
    T = msm;
    uint32_t nchunks = 65536 / b.nslots;  // 1024 waves (16384 lanes: C5's 157-round chains, 8.5 ms)
    if (nchunks < 1) nchunks = 1;
    if (nchunks > b.R) nchunks = b.R;
    uint32_t chunk = (b.R + nchunks - 1) / nchunks;
    nchunks = (b.R + chunk - 1) / chunk;
    RET(wsT(S_KP, (size_t)b.nslots * nchunks, &Kp));
    RET(wsT(S_TMP, (size_t)b.nslots * nchunks, &tmp));
    RET(launch("k_key_accum", k_key_accum, b.nslots * nchunks, 128, st, b.R, b.nslots, chunk, nchunks,
               (const uint32_t*)cell, (const uint8_t*)active, (const G2JStore*)A, Kp));
    RET(reduce_rows(Kp, tmp, b.nslots, nchunks, st));  // -C_s = Kp[s]
    K = Kp;
    HIPCHK(hipStreamWaitEvent(st, c.kc_join, 0));
  }
  const uint32_t npairs = b.nslots + (b.nslots > 1 ? 2u : 1u);
  // the batched subgroup check's window sums ride in the Miller launch (extra workgroups); k_final_coop folds
  // their verdict (flag[2]) into the batch's
  const uint32_t nsub = batched_sub ? MSM_WT * (b.nslots > 1 ? b.nslots : 1u) : 0u;
  RET(launch("k_pair_miller_coop", k_pair_miller_coop, 128 * (npairs + nsub), 128, st, b.nslots, seed,
             b.keys, K, T, (const G1AStore*)Xc, Kc, f, npairs, (const G2JStore*)win, flag + 2));
  RET(launch("k_final_coop", k_final_coop, 128, 128, st, npairs, (const Fp12*)f, flag, (const uint32_t*)flag + 2));
  // isolated items present?  The per-item pass decides on the device (no host round trip), so a batch
  // is one stream-ordered sequence of launches.
  HIPCHK(hipMemsetAsync(flag + 1, 0, 4, st));
  RET(launch("k_any", k_any, N, 256, st, N, (const uint8_t*)iso, flag + 1));
  if (!b.item_pass) {
    out->seed = seed;
    out->flag = flag;
    out->iso = iso;
    out->batched_sub = batched_sub;
    return 0;
  }
  if (b.nslots == 1 && b.k == 1 && !b.item_slot) {
    // one key, one item per round (VerifyBeacon / VerifyRecovered): a failed batch isolates its bad rounds by group
    // tests across rounds (xr.h), enqueued whole and decided on the device, so asynchronous batches stay asynchronous
    // (on a tail stream: the workspace of that stream, shared by the sets it serves)
    struct PoolGuard {
      explicit PoolGuard(int p) { g_ctx.xr_pool = p; }
      ~PoolGuard() { g_ctx.xr_pool = -1; }
    } guard(tst ? cur_set().tail_idx : -1);
    for (uint32_t i0 = 0; i0 < N; i0 += kXrSeg)
      RET(xr_isolate(i0, std::min(kXrSeg, N - i0), flag, seed, b.keys, b.Q, b.S, b.status, st));
  } else {
    // several keys (VerifyPartial, a blocking entry point): the items the equation did not decide -- every decoded
    // item of a failed batch, the isolated ones of a passed batch -- take the group-test passes of checks.h (groups of
    // up to GRP items of a round, then every failed group's members alone; t = k + 1: no round stops early)
    uint8_t* fin;
    uint32_t* inc;
    RET(wsT(S_FIN, N, &fin));
    RET(wsT(S_INC, 4, &inc));
    HIPCHK(hipMemsetAsync(inc, 0, 4, st));
    RET(launch("k_window_fin", k_window_fin, N, 256, st, b.R, b.k, 0u, b.k, (const uint32_t*)flag, (const uint8_t*)iso,
               (const uint8_t*)b.status, b.status, fin, inc));
    uint32_t inc_h = 0;
    HIPCHK(hipMemcpyAsync(&inc_h, inc, 4, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    if (inc_h)
      RET(prefix_pass(b.R, b.k, b.k + 1, 1, seed, b.keys, b.item_slot, b.Q, b.S, b.status, fin, batched_sub, st));
  }
  RET(launch("k_count_fallback", k_count_fallback, 1, 64, st, (const uint32_t*)flag, g_ctx.fallbacks));
  return 0;
}

// The group key of the single-key paths, decoded once per distinct key and shared by the workspace sets:
// decompression + [r]P subgroup check is a ~1.5k-Fp-multiplication single-lane job.
int decode_key(const uint8_t* pk48_host, hipStream_t st, G1AStore** keys, uint8_t** key_status) {
  Ctx& c = g_ctx;
  if (!c.pk_dev) {
    HIPCHK(hipMalloc(&c.pk_dev, sizeof(G1AStore)));
    HIPCHK(hipMalloc(&c.pk_status, 16));
    HIPCHK(hipMalloc(&c.pk_raw, 48));
    HIPCHK(hipEventCreateWithFlags(&c.pk_ready, hipEventDisableTiming));
  }
  *keys = c.pk_dev;
  *key_status = c.pk_status;
  if (c.pk_valid && memcmp(c.pk_bytes, pk48_host, 48) == 0) {
    // a cross-stream wait puts a barrier in the stream's hardware queue: only while the decode is still running
    const hipError_t q = hipEventQuery(c.pk_ready);
    if (q == hipErrorNotReady) HIPCHK(hipStreamWaitEvent(st, c.pk_ready, 0));
    else HIPCHK(q);
    return 0;
  }
  // a previous key may still be in use by batches in flight on other sets
  for (Set& x : c.sets)
    if (x.busy) {
      HIPCHK(hipEventSynchronize(x.done));
      x.busy = false;
    }
  HIPCHK(hipMemcpyAsync(c.pk_raw, pk48_host, 48, hipMemcpyHostToDevice, st));
  RET(launch("k_decode_g1", k_decode_g1, 1, 64, st, 1u, (const uint8_t*)c.pk_raw, c.pk_dev, c.pk_status));
  HIPCHK(hipEventRecord(c.pk_ready, st));
  memcpy(c.pk_bytes, pk48_host, 48);
  c.pk_valid = true;
  return 0;
}

// out[i] = 1 / vals[i] (0 for 0) for n Fp values on the device: Montgomery's trick over chunks of BINV_C, a tree of
// chunk products, one safegcd inversion at the root (phases.h k_binv_*)
int batch_inv_chunked(uint32_t n, const Fp* vals, Fp* out, hipStream_t st, Slot slot);
int batch_inv(uint32_t n, const Fp* vals, Fp* out, hipStream_t st, bool alt) {
  constexpr uint32_t PER = BINV_T * BINV_K;
  if (n <= BINV_T * BINV_R) return launch("k_binv_blk_root", k_binv_blk_root, BINV_T, BINV_T, st, n, vals, out);
  // block tree (phases.h k_binv_blk_*): per block of PER values a root; the roots by the chunked form
  const uint32_t nb = (n + PER - 1) / PER;
  Fp *pre, *roots, *rinv;
  RET(wsT(alt ? S_BINV2_PRE : S_BINV_PRE, n, &pre));
  RET(wsT(alt ? S_BINV2_ROOTS : S_BINV_ROOTS, 2 * (size_t)nb, &roots));
  rinv = roots + nb;
  RET(launch("k_binv_blk_up", k_binv_blk_up, nb * BINV_T, BINV_T, st, n, vals, pre, roots));
  if (nb <= BINV_T * BINV_R)
    RET(launch("k_binv_blk_root", k_binv_blk_root, BINV_T, BINV_T, st, nb, (const Fp*)roots, rinv));
  else
    RET(batch_inv_chunked(nb, roots, rinv, st, alt ? S_BINV2 : S_BINV));  // n > 2M values (its own slot: no reentry)
  return launch("k_binv_blk_down", k_binv_blk_down, nb * BINV_T, BINV_T, st, n, vals, (const Fp*)pre, (const Fp*)rinv,
                out);
}
int batch_inv_chunked(uint32_t n, const Fp* vals, Fp* out, hipStream_t st, Slot slot) {
  std::vector<uint32_t> sizes{n};
  while (sizes.back() > BINV_C) sizes.push_back((sizes.back() + BINV_C - 1) / BINV_C);
  const size_t L = sizes.size();
  size_t total = 0;
  for (size_t l = 0; l < L; ++l) total += 3 * (size_t)sizes[l];
  Fp* buf;
  RET(wsT(slot, total, &buf));
  // level l: in[l] (the values), pre[l], inv[l] (their inverses); in[0] = vals, inv[0] = out
  std::vector<const Fp*> in(L);
  std::vector<Fp*> pre(L), inv(L);
  Fp* q = buf;
  for (size_t l = 0; l < L; ++l) {
    pre[l] = q;
    q += sizes[l];
    inv[l] = l == 0 ? out : q;
    q += sizes[l];
    in[l] = l == 0 ? vals : q;
    q += sizes[l];
  }
  for (size_t l = 0; l + 1 < L; ++l)
    RET(launch("k_binv_up", k_binv_up, (sizes[l] + BINV_C - 1) / BINV_C, 128, st, sizes[l], in[l], pre[l],
               (Fp*)in[l + 1]));
  RET(launch("k_binv_root", k_binv_root, 1, 64, st, sizes[L - 1], in[L - 1], inv[L - 1]));
  for (size_t l = L - 1; l-- > 0;)
    RET(launch("k_binv_down", k_binv_down, (sizes[l] + BINV_C - 1) / BINV_C, 128, st, sizes[l], in[l],
               (const Fp*)pre[l], (const Fp*)inv[l + 1], inv[l]));
  return 0;
}

// The current DST and its expand_message_xmd tail on the device (blocking upload after a DST change: batches
// in flight keep reading the old bytes until they finish, so they are waited for first).
int ensure_dst() {
  Ctx& c = g_ctx;
  if (c.dst_dev_valid) return 0;
  for (Set& x : c.sets)
    if (x.busy) {
      HIPCHK(hipEventSynchronize(x.done));
      x.busy = false;
    }
  if (!c.d_dst) HIPCHK(hipMalloc(&c.d_dst, 256));
  if (!c.d_xmd) HIPCHK(hipMalloc(&c.d_xmd, sizeof(XmdTail)));
  xmd_tail_build(c.xmd, c.dst.data(), (uint32_t)c.dst.size());
  HIPCHK(hipMemcpy(c.d_dst, c.dst.data(), c.dst.size(), hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(c.d_xmd, &c.xmd, sizeof(XmdTail), hipMemcpyHostToDevice));
  c.dst_dev_valid = true;
  return 0;
}

int hash_rounds(uint32_t R, const uint8_t* d_msgs, uint32_t msg_len, hipStream_t st, G2JStore** Q) {
  uint8_t* d_dst;
  RET(ensure_dst());
  d_dst = g_ctx.d_dst;
  RET(wsT(S_Q, R, Q));
  // phases.h: two maps per round, every exponentiation through k_exp_pm3d4
  const uint32_t M = 2 * R;
  H2cMap* hs;
  Fp *ein, *eout;
  G2JStore* iso;
  RET(wsT(S_H2CST, M, &hs));
  RET(wsT(S_EIN, M, &ein));
  RET(wsT(S_EOUT, M, &eout));
  RET(wsT(S_ISOPT, M, &iso));
  Fp *nv, *nvinv;
  RET(wsT(S_NV, R, &nv));
  RET(wsT(S_NVINV, R, &nvinv));
  RET(launch("k_h2c_p1a", k_h2c_p1a, R, 128, st, R, d_msgs, msg_len, (const uint8_t*)d_dst, (uint32_t)g_ctx.dst.size(),
             (const XmdTail*)g_ctx.d_xmd, hs, nv));
  RET(batch_inv(R, nv, nvinv, st));
  RET(launch("k_h2c_p1b", k_h2c_p1b, R, 128, st, R, hs, (const Fp*)nvinv, ein));
  RET(launch("k_exp_pm3d4", k_exp_pm3d4, M, 128, st, M, (const Fp*)ein, eout));
  RET(launch("k_h2c_p2", k_h2c_p2, M, 128, st, M, hs, ein, (const Fp*)eout));
  RET(launch("k_exp_pm3d4", k_exp_pm3d4, M, 128, st, M, (const Fp*)ein, eout));
  RET(launch("k_h2c_p3", k_h2c_p3, M, 128, st, M, (const H2cMap*)hs, (const Fp*)ein, (const Fp*)eout, iso));
  RET(launch("k_h2c_p4a", k_h2c_p4a, R, 128, st, R, (const G2JStore*)iso, *Q, nv));
  RET(batch_inv(R, nv, nvinv, st));
  return launch("k_h2c_p4b", k_h2c_p4b, R, 128, st, R, *Q, (const Fp*)nvinv);
}

// bls.Verify batch against one key, everything device-resident
int verify_single_key(const uint8_t* pk48_host, uint32_t n, const uint8_t* d_msgs, uint32_t msg_len,
                      const uint8_t* d_sigs, uint8_t* d_status, uint64_t seed, hipStream_t st, hipStream_t tst = nullptr) {
  G1AStore* keys;
  uint8_t* kst;
  G2JStore* Q;
  G2AStore* S;
  RET(decode_key(pk48_host, st, &keys, &kst));
  RET(hash_rounds(n, d_msgs, msg_len, st, &Q));
  RET(wsT(S_S, n, &S));
  Batch b{n, 1, 1, Q, keys, kst, nullptr, d_sigs, 96, 0, S, d_status, d_msgs, msg_len, pk48_host, 48};
  RET(batch_verify(b, seed, st, nullptr, tst));
  return 0;
}

// X_i = PubPoly.Eval(i) for the distinct indices idx (slot order), from the context cache when the commits
// and indices are those of the previous call
int poly_keys(const uint8_t* commits48, uint32_t t, const std::vector<uint32_t>& idx, hipStream_t st, G1AStore** keys,
              uint8_t** kst) {
  Ctx& c = g_ctx;
  const uint32_t nslots = (uint32_t)idx.size();
  if (c.poly_valid && c.poly_idx == idx && c.poly_commits.size() == (size_t)t * 48 &&
      memcmp(c.poly_commits.data(), commits48, (size_t)t * 48) == 0) {
    HIPCHK(hipStreamWaitEvent(st, c.poly_ready, 0));
    *keys = c.poly_keys;
    *kst = c.poly_kst;
    return 0;
  }
  // the multi-key entry points are blocking, so no batch in flight reads the cached keys
  c.poly_valid = false;
  if (!c.poly_ready) HIPCHK(hipEventCreateWithFlags(&c.poly_ready, hipEventDisableTiming));
  if (c.poly_cap < nslots) {
    if (c.poly_keys) HIPCHK(hipFree(c.poly_keys));
    if (c.poly_kst) HIPCHK(hipFree(c.poly_kst));
    c.poly_keys = nullptr;
    c.poly_kst = nullptr;
    c.poly_cap = 0;
    HIPCHK(hipMalloc(&c.poly_keys, sizeof(G1AStore) * nslots));
    HIPCHK(hipMalloc(&c.poly_kst, nslots));
    c.poly_cap = nslots;
  }
  uint8_t *d_c, *d_cst;
  G1AStore* cA;
  uint32_t* d_slotidx;
  RET(upload(S_IN0, commits48, (size_t)t * 48, &d_c, st));
  RET(wsT(S_COMMITS, t, &cA));
  RET(wsT(S_COMMITST, t, &d_cst));
  RET(launch("k_decode_g1", k_decode_g1, t, 64, st, t, (const uint8_t*)d_c, cA, d_cst));
  RET(upload(S_SLOTIDX, idx.data(), nslots, &d_slotidx, st));
  RET(launch("k_pubpoly_eval", k_pubpoly_eval, nslots, 64, st, nslots, t, (const G1AStore*)cA, (const uint8_t*)d_cst,
             (const uint32_t*)d_slotidx, c.poly_keys, c.poly_kst, (uint8_t*)nullptr));
  HIPCHK(hipEventRecord(c.poly_ready, st));
  c.poly_commits.assign(commits48, commits48 + (size_t)t * 48);
  c.poly_idx = idx;
  c.poly_valid = true;
  *keys = c.poly_keys;
  *kst = c.poly_kst;
  return 0;
}

// Key slots of a VerifyPartial / Recover batch over R rounds x k partials (d_p: device records).  An index enters the
// batch equation as its own key set only if it occurs in at least 1/8 of the rounds' first w partials (the batch's
// items), and at most kMaxSlots of them (most frequent first): each set costs an MSM bucket array, a column of the
// (round, key) cell map and possibly a correction pairing, so a signer that sends a fresh index every round must
// not get one per index.  Items of the other indices, and every index seen only beyond the window, are checked on
// their own (their verdicts stay exact).  Counts and first positions come from the device (k_index_scan: 2 x 256 KB
// back to the host instead of a host pass over the partials); the slot table goes back up (256 KB).  keys: X_i =
// PubPoly.Eval(i) for every distinct index of the R x k items; item_slot: every item's slot.
int plan_slots(const uint8_t* commits48, uint32_t t, uint32_t R, uint32_t k, uint32_t w, const uint8_t* d_p,
               hipStream_t st, G1AStore** keys, uint8_t** kst, uint32_t** d_itemslot, uint32_t* nslots_out) {
  const size_t N = (size_t)R * k;
  uint32_t *d_cnt, *d_first;
  RET(wsT(S_IDXCNT, 65536, &d_cnt));
  RET(wsT(S_IDXFIRST, 65536, &d_first));
  HIPCHK(hipMemsetAsync(d_cnt, 0, 65536 * 4, st));
  HIPCHK(hipMemsetAsync(d_first, 0xff, 65536 * 4, st));
  RET(launch("k_index_scan", k_index_scan, (uint32_t)N, 256, st, (uint32_t)N, k, w, d_p, d_cnt, d_first));
  std::vector<uint32_t> count(65536), first(65536);
  HIPCHK(hipMemcpyAsync(count.data(), d_cnt, 65536 * 4, hipMemcpyDeviceToHost, st));
  HIPCHK(hipMemcpyAsync(first.data(), d_first, 65536 * 4, hipMemcpyDeviceToHost, st));
  HIPCHK(hipStreamSynchronize(st));
  std::vector<uint32_t> distinct;
  for (uint32_t idx = 0; idx < 65536; ++idx)
    if (first[idx] != ~0u) distinct.push_back(idx);
  std::stable_sort(distinct.begin(), distinct.end(), [&](uint32_t a, uint32_t b) { return count[a] > count[b]; });
  constexpr uint32_t kMaxSlots = 1024;
  uint32_t nslots = 0;
  while (nslots < distinct.size() && nslots < kMaxSlots && count[distinct[nslots]] > 0 &&
         (nslots == 0 || (size_t)count[distinct[nslots]] * 8 >= R))
    ++nslots;
  if (nslots == 0) nslots = 1;  // (no item in the window: one empty key set)
  // slots in first-occurrence order within each class (batched, alone), so the usual batch keeps the
  // input's index order
  std::vector<uint32_t> slot_idx(distinct.begin(), distinct.begin() + std::min<size_t>(nslots, distinct.size()));
  std::vector<uint32_t> alone(distinct.begin() + slot_idx.size(), distinct.end());
  auto by_first = [&](uint32_t a, uint32_t b) { return first[a] < first[b]; };
  std::sort(slot_idx.begin(), slot_idx.end(), by_first);
  std::sort(alone.begin(), alone.end(), by_first);
  slot_idx.insert(slot_idx.end(), alone.begin(), alone.end());
  std::vector<int32_t> slot_of(65536, -1);
  for (size_t q = 0; q < slot_idx.size(); ++q) slot_of[slot_idx[q]] = (int32_t)q;
  int32_t* d_slotof;
  RET(poly_keys(commits48, t, slot_idx, st, keys, kst));
  RET(upload(S_SLOTOF, slot_of.data(), 65536, &d_slotof, st));
  RET(wsT(S_ITEMSLOT, N, d_itemslot));
  RET(launch("k_item_slots", k_item_slots, (uint32_t)N, 256, st, (uint32_t)N, d_p, (const int32_t*)d_slotof,
             *d_itemslot));
  *nslots_out = nslots;
  return 0;
}

// VerifyPartial over R rounds x k partials (messages d_m and 98 B records d_p in device memory): keys X_i =
// PubPoly.Eval(i) for every distinct index; the statuses are left in *d_status (stream order)
int verify_partials_dev(const uint8_t* commits48, uint32_t t, uint32_t R, const uint8_t* d_m, uint32_t msg_len,
                        uint32_t k, const uint8_t* d_p, uint64_t seed, hipStream_t st, uint8_t** d_status) {
  const size_t N = (size_t)R * k;
  uint8_t* kst;
  G1AStore* keys;
  uint32_t *d_itemslot, nslots;
  RET(plan_slots(commits48, t, R, k, k, d_p, st, &keys, &kst, &d_itemslot, &nslots));
  G2JStore* Q;
  G2AStore* S;
  RET(hash_rounds(R, d_m, msg_len, st, &Q));
  RET(wsT(S_S, N, &S));
  RET(wsT(S_STATUS, N, d_status));
  Batch b{R, k, nslots, Q, keys, kst, d_itemslot, d_p, 98, 2, S, *d_status, d_m, msg_len, commits48, (size_t)t * 48};
  return batch_verify(b, seed, st);
}

// Recover's per-item pass over the examined prefix (on the per-item stream, ordered after and before the batch's
// stream).  Recover (kyber tbls.Recover) checks the partials of a round in input order and stops at the t-th valid
// one, so only the items up to that point need a verdict: about t / (1 - corrupted fraction) of the k.  Passes grow
// the prefix by each round's deficit; the last takes every unverified item before the t-th valid one, so the
// statuses Recover reads are exact.  Up to GRP fresh items of a round are checked together (kernels.h
// verify_group); the members of a failed group, and everything in the last pass, are checked alone.  DG_GROUP=1
// checks every item alone.  fin: FIN_DONE for the final verdicts, FIN_PENDING for the rest.
// The pairing-check pipeline of checks.h: per-check workspace of the current set, sized for the G checks of the launch
// at hand (grow-only slots: a small call allocates little).
struct CkBufs {
  CkState* st;
  CkLine* l2;
  Fp12 *F, *F2, *T0, *T1, *A;
  Fp* nv;
  CycC* sn;
  uint8_t *zero, *good;
  uint32_t* zl;  // CK_NEXP work lists of k_ck_explain, (G + 1) words each: [0] = count, then the checks
  // the split G2 sums of Recover's group checks (checks.h k_ck_tab_* / k_ck_sac / k_ck_bfin)
  uint4* T4;
  uint8_t *tinf, *g2m;
  RsDigits* dig;
  Fp *tden, *bn;
  G2JStore* bj;
};
int ck_bufs(CkBufs& b, size_t G, bool group_sums, bool lines = true) {
  RET(wsT(S_CK_ST, G, &b.st));
  b.l2 = nullptr;
  if (lines) RET(wsT(S_CK_L2, (size_t)CK_STEPS * G, &b.l2));  // (not for the isolation: xr.h k_xg_miller)
  RET(wsT(S_CK_F, 2 * G, &b.F));  // (two pairs' values per check for xr.h k_xg_miller)
  RET(wsT(S_CK_F2, G, &b.F2));
  RET(wsT(S_CK_T0, G, &b.T0));
  RET(wsT(S_CK_T1, G, &b.T1));
  RET(wsT(S_CK_A, G, &b.A));
  RET(wsT(S_CK_NV, CK_NPOW * G, &b.nv));
  RET(wsT(S_CK_SN, CK_NPOW * G, &b.sn));
  RET(wsT(S_CK_ZERO, G, &b.zero));
  RET(wsT(S_CK_GOOD, G, &b.good));
  RET(wsT(S_CK_ZL, CK_NEXP * (G + 1), &b.zl));
  if (group_sums) {
    RET(wsT(S_CK_T4, 8 * RC_Q * G, &b.T4));
    RET(wsT(S_CK_TINF, 8 * G, &b.tinf));
    RET(wsT(S_CK_DIG, G, &b.dig));
    RET(wsT(S_CK_TDEN, 6 * G, &b.tden));
    RET(wsT(S_CK_BJ, G, &b.bj));
    RET(wsT(S_CK_BN, 2 * G, &b.bn));
    RET(wsT(S_CK_G2M, G, &b.g2m));
  }
  return 0;
}
// X^z (pairing.h cyc_exp_z) times the hard part's next factor: the compressed chain (k_ck_expsq2), the decompressed
// product with the six norms inverted in the lane (k_ck_expdec), the uncompressed chain for the lanes with a zero
// denominator (k_ck_explain over work list z, CK_EXPLAIN_LANES lanes: it is rare); out = X^z op(Y) (Y may be null)
int ck_expz(uint32_t z, uint32_t G, const uint32_t* gcnt, const Fp12* X, const Fp12* Y, uint32_t nfrob, uint32_t conj,
            Fp12* out, const CkBufs& b, hipStream_t st) {
  uint32_t* zl = b.zl + (size_t)z * (G + 1);
  // two lanes per check everywhere (C5 15.3 -> 15.6 k: the one-lane form spilled 79 VGPRs)
  RET(launch("k_ck_expsq2", k_ck_expsq2, 2 * G, 64, st, G, gcnt, X, b.sn, b.nv, b.zero, zl));
  RET(launch("k_ck_expdec", k_ck_expdec, G, 64, st, G, gcnt, (const CycC*)b.sn, b.nv, (const uint8_t*)b.zero, Y, nfrob,
             conj, out));
  return launch("k_ck_explain", k_ck_explain, CK_EXPLAIN_LANES, 64, st, (const uint32_t*)zl, X, Y, nfrob, conj, out);
}
// The final exponentiation of the checks b.st[0..G) from their Miller values b.F (two != 0: the two pairs' values F[g],
// F[G + g], multiplied first) -> b.good: k_ck_easy, five x^z with their next factors, k_ck_final.  Every kernel is one
// lane per check without exchange, so gcnt (device, may be null) gates the lanes of a launch sized for G.
int run_final(uint32_t G, const uint32_t* gcnt, const CkBufs& b, hipStream_t st, uint32_t two) {
  RET(launch("k_ck_easy", k_ck_easy, G, 64, st, G, gcnt, two, (const Fp12*)b.F, b.F2, b.zl));
  // hard part (final_exp_cubed): t0 = f2^z conj(f2), t1 = t0^z conj(t0), a = t1^z frob(t1),
  // b = (a^z)^z frob^2(a) conj(a), c = f2^3, result b c
  RET(ck_expz(0, G, gcnt, b.F2, b.F2, 0, 1, b.T0, b, st));
  RET(ck_expz(1, G, gcnt, b.T0, b.T0, 0, 1, b.T1, b, st));
  RET(ck_expz(2, G, gcnt, b.T1, b.T1, 1, 0, b.A, b, st));
  RET(ck_expz(3, G, gcnt, b.A, nullptr, 0, 0, b.T0, b, st));
  RET(ck_expz(4, G, gcnt, b.T0, b.A, 2, 0, b.T1, b, st));
  return launch("k_ck_final", k_ck_final, G, 64, st, G, gcnt, (const CkState*)b.st, (const Fp12*)b.T1,
                (const Fp12*)b.A, (const Fp12*)b.F2, b.good);
}
// The checks b.st[0..G) of Recover's / VerifyPartial's passes (pair 0: (a, the lines rl[s R + round]), pair 1: (-g1, b))
// -> b.good: the (-g1, b) lines, the Miller values (both pairs in one lane), the final exponentiation
int run_checks(uint32_t G, uint32_t R, const CkLine* rl, const CkBufs& b, hipStream_t st) {
  RET(launch("k_ck_lines2", k_ck_lines2, G, 64, st, G, (const uint32_t*)nullptr, (const CkState*)b.st, b.l2));
  RET(launch("k_ck_miller", k_ck_miller, G, 64, st, G, (const uint32_t*)nullptr, R, (const CkState*)b.st, rl,
             (const CkLine*)b.l2, b.F));
  return run_final(G, nullptr, b, st, 0u);
}
// Recover's / VerifyPartial's group checks glist[4 + 4 (off + g)] of one pass (G <= CK_CHUNK): members and weighted
// sums, the checks, the verdicts
int check_chunk(uint32_t G, uint32_t off, const uint32_t* glist, uint32_t k, uint32_t R, const uint64_t* seed,
                const G1AStore* keys, const uint32_t* item_slot, const uint8_t* hinf, const CkLine* rl, const G2AStore* S,
                uint8_t* status, uint8_t* fin, uint32_t subgroup, hipStream_t st) {
  CkBufs b;
  RET(ck_bufs(b, G, true));
  if (subgroup) RET(launch("k_ck_sub", k_ck_sub, 4 * G, 64, st, G, off, glist, (const G2AStore*)S, status, fin));
  RET(launch("k_ck_prep", k_ck_prep, G, 64, st, G, off, glist, k, seed, keys, item_slot, hinf, S, status, fin, 0u,
             g_ctx.gcount, b.st, b.g2m, b.dig));
  Fp *den = b.tden, *dinv = b.tden + 3 * (size_t)G;
  for (uint32_t l = 0; l < 3; ++l) {
    RET(launch("k_ck_tab_den", k_ck_tab_den, 3 * G, 64, st, l, G, (const CkState*)b.st, (const uint8_t*)b.g2m, S, b.T4,
               b.tinf, den));
    RET(batch_inv(3 * G, den, dinv, st));
    RET(launch("k_ck_tab_add", k_ck_tab_add, 3 * G, 64, st, l, G, (const CkState*)b.st, (const uint8_t*)b.g2m, S, b.T4,
               b.tinf, (const Fp*)dinv));
  }
  RET(launch("k_ck_sac", k_ck_sac, G, 64, st, G, (const uint8_t*)b.g2m, (const RsDigits*)b.dig, (const uint4*)b.T4,
             (const uint8_t*)b.tinf, b.bj, b.bn));
  RET(batch_inv(G, b.bn, b.bn + G, st));
  RET(launch("k_ck_bfin", k_ck_bfin, G, 64, st, G, (const uint8_t*)b.g2m, (const G2JStore*)b.bj, (const Fp*)(b.bn + G),
             hinf, b.st));
  RET(run_checks(G, R, rl, b, st));
  return launch("k_ck_verdict", k_ck_verdict, G, 128, st, G, (const CkState*)b.st, (const uint8_t*)b.good, status, fin);
}

// Cross-round isolation of a failed single-key batch (xr.h): items [i0, i0 + n) of the batch (its status, decoded S,
// uncleared hashes Q, the group key keys[0]), two levels of group tests on the device, no host round trip; after a
// passed batch every launch returns at once.  At most kXrSeg items per run; a check's workspace is ~5 KB (no line
// table: k_xg_miller computes each pair's lines in the lane), so a segment's worst case -- every round a single check --
// is ~0.7 GB, held once per tail stream.
uint32_t xr_qpg() {  // quads per level-1 group (DG_XR_QPG: a test hook for the level shapes)
  static const uint32_t v = (uint32_t)std::max(1, std::min(64, env_int("DG_XR_QPG", (int)XR_QPG)));
  return v;
}
int xr_isolate(uint32_t i0, uint32_t n, const uint32_t* flag, const uint64_t* seed, const G1AStore* keys,
               const G2JStore* Q, const G2AStore* S, uint8_t* status, hipStream_t st) {
  const uint32_t qpg = xr_qpg(), nqmax = (n + 3) / 4, G1 = (nqmax + qpg - 1) / qpg;
  uint32_t *cnt, *cand, *l3;
  G2JStore *QS, *HS;
  uint4* T4;
  uint8_t* tinf;
  CkBufs b;
  RET(wsT(S_XR_CNT, XR_NCNT, &cnt));
  RET(wsT(S_XR_CAND, n, &cand));
  RET(wsT(S_XR_L3, n, &l3));
  RET(wsT(S_XR_QS, 2 * (size_t)nqmax, &QS));
  RET(wsT(S_XR_T4, (size_t)8 * RC_Q * 2 * nqmax, &T4));
  RET(wsT(S_XR_TINF, (size_t)8 * 2 * nqmax, &tinf));
  RET(wsT(S_XR_HS, n, &HS));
  RET(ck_bufs(b, n, false, false));
  RET(launch("k_xg_sub", k_xg_sub, n, 64, st, i0, n, flag, S, status, cnt));
  RET(launch("k_xg_cand", k_xg_cand, n, 256, st, i0, n, flag, (const uint8_t*)status, cand, cnt));
  RET(launch("k_xq_sum", k_xq_sum, 2 * nqmax, 64, st, nqmax, qpg, seed, cnt, (const uint32_t*)cand, Q, S, T4, tinf, QS));
  for (uint32_t level : {1u, 3u}) {
    const uint32_t G = level == 1 ? G1 : n, Gp = (G + 63) & ~63u;
    const uint32_t* gcnt = cnt + level;
    RET(launch("k_xg_prep", k_xg_prep, G, 64, st, level, G, gcnt, (const uint32_t*)cnt, qpg, (const uint32_t*)l3,
               (const G2JStore*)QS, Q, S, keys, b.st, HS));
    RET(launch("k_xg_heff", k_xg_heff, G, 64, st, G, gcnt, HS, b.st));
    RET(launch("k_xg_miller", k_xg_miller, 2 * Gp, 64, st, G, gcnt, (const G2JStore*)HS, (const CkState*)b.st, b.F));
    RET(run_final(G, gcnt, b, st, 1u));
    RET(launch("k_xg_verdict", k_xg_verdict, G, 128, st, level, G, gcnt, qpg, cnt, (const uint8_t*)b.good,
               (const uint32_t*)cand, l3, status, g_ctx.xrcount));
  }
  return 0;
}

// The pass schedule of the pipeline: DG_CK_PASSES passes with speculative margins (DG_CK_MARGIN0 in the first,
// DG_CK_MARGIN in the others), then the final pass over every unverified share before the t-th valid one.  Every pass
// costs at least the latency of one check (a lane's Miller loop alone is ~13 ms), however few checks it holds.
int ck_passes() {
  static const int v = env_int("DG_CK_PASSES", 8);
  return v < 0 ? 0 : v;
}
uint32_t ck_margin(int which) {
  static const int m0 = env_int("DG_CK_MARGIN0", 6), m = env_int("DG_CK_MARGIN", 2);
  return (uint32_t)(which == 0 ? m0 : m);
}

// The per-item pass of a multi-key batch (Recover's examined prefix, VerifyPartial's isolated or failed items) on the
// batch's own stream: H_r's lines once per round (k_ck_round_lines), then `passes` passes of group tests with
// speculative margins and a final pass of single checks over every unverified item before the t-th valid one of its
// round (t > k: every unverified item).  Per pass the group list is built on the device and its size read back, so
// the pipeline runs over chunks of at most CK_CHUNK checks.  Statuses exact at the end; fin: FIN_DONE for the final
// verdicts, FIN_PENDING for the rest (the seed's weights rho_i: kernels.h group_combine).
int prefix_pass(uint32_t R, uint32_t k, uint32_t t, int passes, const uint64_t* seed, const G1AStore* keys,
                const uint32_t* item_slot, const G2JStore* Q, const G2AStore* S, uint8_t* status, uint8_t* fin,
                uint32_t subgroup, hipStream_t st) {
  const size_t N = (size_t)R * k;
  CkLine* rl;
  uint8_t* hinf;
  uint32_t* glist;
  RET(wsT(S_CK_RL, (size_t)CK_STEPS * R, &rl));
  RET(wsT(S_CK_HINF, R, &hinf));
  RET(wsT(S_LIST, 4 * (N + 1), &glist));
  RET(launch("k_ck_round_lines", k_ck_round_lines, R, 64, st, R, Q, rl, hinf));
  const uint32_t grp = group_size();
  for (int pass = 0; pass <= passes; ++pass) {
    HIPCHK(hipMemsetAsync(glist, 0, 4, st));
    const uint32_t margin = grp < 2 ? 0u : (pass == 0 ? ck_margin(0) : ck_margin(1));
    RET(launch("k_prefix_groups", k_prefix_groups, R, 128, st, R, k, t, pass == passes ? 1u : 0u, grp, margin,
               (const uint8_t*)status, (const uint8_t*)fin, glist));
    uint32_t G = 0;
    HIPCHK(hipMemcpyAsync(&G, glist, 4, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    static const bool trace = getenv("DG_CK_TRACE") != nullptr;  // diagnostics: checks per pass
    if (trace) fprintf(stderr, "[dg] prefix pass %d: %u checks\n", pass, G);
    for (uint32_t off = 0; off < G; off += CK_CHUNK)
      RET(check_chunk(std::min(G - off, CK_CHUNK), off, glist, k, R, seed, keys, item_slot, hinf, rl, S, status, fin,
                      subgroup, st));
  }
  return 0;
}

// Recover's VerifyPartial verdicts, examined prefix first.  The batch equation covers the first w = min(t, k)
// partials of every round (gathered into an R x w table).  When it holds and every window item decoded -- every
// round of a valid chain -- each round's first t partials are valid, which is all kyber's Recover examines
// (beacon/beacon.go:488): the other k - w are never decoded.  Otherwise the items beyond the window are decoded
// (beside the window's into the R x k tables) and the per-item pass decides every verdict of the examined prefix,
// with coefficients bound to all R x k items.  Outputs: the R x k statuses and decoded sigmas (items beyond the
// window of a complete round are left unset: Recover never reads them).
int recover_windowed(const uint8_t* commits48, uint32_t t, uint32_t R, const uint8_t* d_m, uint32_t msg_len, uint32_t k,
                     const uint8_t* d_p, uint64_t seed, hipStream_t st, uint8_t** d_status, G2AStore** d_S) {
  const uint32_t w = t < k ? t : k;
  const size_t N = (size_t)R * k, Nw = (size_t)R * w;
  if (N * 49 > 0x7fffffffull) return fail(DG_E_ARG, "Recover batch too large (rounds x k >= 2^31 / 49)");
  uint8_t* kst;
  G1AStore* keys;
  uint32_t *d_itemslot, nslots;
  RET(plan_slots(commits48, t, R, k, w, d_p, st, &keys, &kst, &d_itemslot, &nslots));
  const uint8_t* d_pw = d_p;
  const uint32_t* d_slotw = d_itemslot;
  if (w < k) {
    uint16_t* pw;
    uint32_t* sw;
    RET(wsT(S_PW, Nw * 49, &pw));
    RET(wsT(S_SLOTW, Nw, &sw));
    RET(launch("k_rows", k_rows<uint16_t>, (uint32_t)(Nw * 49), 256, st, R, w, 49u, k, 0u, w, 0u, (const uint16_t*)d_p, pw));
    RET(launch("k_rows", k_rows<uint32_t>, (uint32_t)Nw, 256, st, R, w, 1u, k, 0u, w, 0u, (const uint32_t*)d_itemslot, sw));
    d_pw = (const uint8_t*)pw;
    d_slotw = sw;
  }
  G2JStore* Q;
  G2AStore* Sw;
  uint8_t* stw;
  RET(hash_rounds(R, d_m, msg_len, st, &Q));
  RET(wsT(S_S, Nw, &Sw));
  RET(wsT(S_STATUS, Nw, &stw));
  Batch bw{R, w, nslots, Q, keys, kst, d_slotw, d_pw, 98, 2, Sw, stw, d_m, msg_len, commits48, (size_t)t * 48};
  bw.item_pass = false;
  BatchOut bo;
  RET(batch_verify(bw, seed, st, &bo));
  // the window's verdicts into the R x k tables
  G2AStore* S;
  uint8_t *status, *fin;
  uint32_t* inc;
  RET(wsT(S_SFULL, N, &S));
  RET(wsT(S_STFULL, N, &status));
  RET(wsT(S_FIN, N, &fin));
  RET(wsT(S_INC, 4, &inc));
  HIPCHK(hipMemsetAsync(inc, 0, 16, st));
  // items beyond the window start as "not examined" (the fast path never decodes them; the slow path overwrites
  // them below), so no status of an earlier batch survives in the reused buffer
  if (w < k) HIPCHK(hipMemsetAsync(status, DG_ST_NOT_EXAMINED_, N, st));
  constexpr uint32_t kQ = sizeof(G2AStore) / 16;
  static_assert(sizeof(G2AStore) % 16 == 0, "G2AStore rows move as uint4");
  RET(launch("k_rows", k_rows<uint4>, (uint32_t)(Nw * kQ), 256, st, R, w, kQ, w, 0u, k, 0u, (const uint4*)Sw, (uint4*)S));
  RET(launch("k_window_fin", k_window_fin, (uint32_t)Nw, 256, st, R, k, 0u, w, bo.flag, bo.iso, (const uint8_t*)stw,
             status, fin, inc));
  uint32_t inc_h = 0;
  HIPCHK(hipMemcpyAsync(&inc_h, inc, 4, hipMemcpyDeviceToHost, st));
  HIPCHK(hipStreamSynchronize(st));
  *d_status = status;
  *d_S = S;
  if (inc_h == 0) return 0;
  // Slow path: decode the items beyond the window (their verdicts are pending until checked)
  const uint64_t* pseed = bo.seed;
  if (w < k) {
    const uint32_t kb = k - w;
    const size_t Nb = (size_t)R * kb;
    uint16_t* pb;
    uint32_t* sb;
    G2AStore* Sb;
    uint8_t *stb, *isob;
    RET(wsT(S_PB, Nb * 49, &pb));
    RET(wsT(S_SLOTB, Nb, &sb));
    RET(launch("k_rows", k_rows<uint16_t>, (uint32_t)(Nb * 49), 256, st, R, kb, 49u, k, w, kb, 0u, (const uint16_t*)d_p, pb));
    RET(launch("k_rows", k_rows<uint32_t>, (uint32_t)Nb, 256, st, R, kb, 1u, k, w, kb, 0u, (const uint32_t*)d_itemslot, sb));
    RET(wsT(S_SB, Nb, &Sb));
    RET(wsT(S_STB, Nb, &stb));
    RET(wsT(S_ISOB, Nb, &isob));
    RET(decode_items((uint32_t)Nb, kb, 0u, (const uint8_t*)pb, 98, 2, sb, kst, Sb, stb, inc + 2, isob,
                     1u - bo.batched_sub, st));
    RET(launch("k_rows", k_rows<uint4>, (uint32_t)(Nb * kQ), 256, st, R, kb, kQ, kb, 0u, k, w, (const uint4*)Sb, (uint4*)S));
    RET(launch("k_window_fin", k_window_fin, (uint32_t)Nb, 256, st, R, k, w, kb, (const uint32_t*)nullptr,
               (const uint8_t*)isob, (const uint8_t*)stb, status, fin, inc + 1));
    // the group tests' coefficients bound to every item they may check
    uint64_t* s2;
    Batch bf{R, k, nslots, Q, keys, kst, d_itemslot, d_p, 98, 2, S, status, d_m, msg_len, commits48, (size_t)t * 48};
    RET(bind_seed(bf, seed ^ 0x77696e646f77ull, st, &s2, S_SEED2));
    pseed = s2;
  }
  RET(prefix_pass(R, k, t, ck_passes(), pseed, keys, d_itemslot, (const G2JStore*)Q, S, status, fin, bo.batched_sub,
                  st));
  return launch("k_count_fallback", k_count_fallback, 1, 64, st, bo.flag, g_ctx.fallbacks);
}

// Recover's divergent rounds (recover.h k_rs_*): the rounds nl[0..Rn) of the blocks whose rounds selected different
// index sets, one sign-aligned joint MSM per round in lanes of RS_G shares, sums into out[r].
int recover_sac(uint32_t R, uint32_t k, uint32_t t, uint32_t Rn, const uint32_t* nl, const uint32_t* d_selidx,
                const uint32_t* d_sel, const uint8_t* d_rst, const G2AStore* d_S, G2JStore* out, hipStream_t st) {
  const size_t n = (size_t)t * Rn;
  if (3 * n > 0x7fffffffull) return fail(DG_E_ARG, "Recover batch too large for the column tables");
  static const uint32_t gs = (uint32_t)std::max(1, std::min(64, env_int("DG_RS_G", (int)RS_G)));
  const uint32_t ngroups = (t + gs - 1) / gs;
  RsDigits* dig;
  uint4* T4;
  uint8_t* pinf;
  Fp *den, *dinv;
  G2JStore* Aps;
  RET(wsT(S_RS_DIG, n, &dig));
  RET(wsT(S_RC_TAB, n * 8 * RC_Q, &T4));
  RET(wsT(S_RC_PINF, n, &pinf));
  RET(wsT(S_RC_DEN, 6 * n, &den));
  dinv = den + 3 * n;
  RET(wsT(S_RC_A, (size_t)ngroups * Rn, &Aps));
  RET(launch("k_rs_digits", k_rs_digits, (uint32_t)n, RS_DIG_NT, st, R, Rn, t, nl, d_selidx, d_rst, dig));
  for (uint32_t l = 0; l < 3; ++l) {
    RET(launch("k_rs_tab_den", k_rs_tab_den, (uint32_t)(3 * n), 128, st, l, R, Rn, k, t, nl, d_rst, d_sel, d_S,
               (const uint4*)T4, pinf, den));
    RET(batch_inv((uint32_t)(3 * n), den, dinv, st));
    RET(launch("k_rs_tab_add", k_rs_tab_add, (uint32_t)(3 * n), 128, st, l, R, Rn, k, t, nl, d_rst, d_sel, d_S, T4,
               (const uint8_t*)pinf, (const Fp*)dinv));
  }
  RET(launch("k_rs_sac", k_rs_sac, ngroups * Rn, 64, st, R, Rn, t, ngroups, gs, nl, d_rst, (const RsDigits*)dig,
             (const uint4*)T4, (const uint8_t*)pinf, Aps));
  return launch("k_rs_combine", k_rs_combine, Rn, 128, st, R, Rn, ngroups, nl, d_rst, (const G2JStore*)Aps, out);
}

// Recover after the VerifyPartial statuses are known (d_st): per round the first t valid partials, xyCommit
// dedupe, Lagrange terms lambda_j S_j, row sums, compression; results copied to the output buffers (host or
// device memory: hipMemcpyDefault).
// Recover's per-round MSM over the uniform blocks (recover.h): lambda / digit schedules per block, the odd-multiple
// tables (affine levels with batch inversions), the four psi-component Straus lanes per round, the combination
// into out[r].  ub: the U uniform blocks that hold an OK round (device).
int recover_msm(uint32_t R, uint32_t k, uint32_t t, uint32_t U, const uint32_t* ub, const uint32_t* ref,
                const uint32_t* d_selidx, const uint32_t* d_sel, const uint8_t* d_rst, const G2AStore* d_S,
                G2JStore* out, hipStream_t st) {
  const uint32_t Ru = U * RC_BLK, maxev = t * RC_EV_PER_SHARE;
  const size_t nel = (size_t)t * Ru;
  if (nel > 0x7fffffffull) return fail(DG_E_ARG, "Recover batch too large for the MSM tables");
  int8_t* naf;
  uint32_t *ev, *hdr;
  uint4 *T4, *D4;
  uint8_t* pinf;
  Fp *den, *dinv;
  G2JStore* A;
  RET(wsT(S_RC_NAF, (size_t)4 * U * t * RC_NAF, &naf));
  RET(wsT(S_RC_EV, (size_t)4 * U * maxev + (size_t)8 * U, &ev));
  hdr = ev + (size_t)4 * U * maxev;
  RET(wsT(S_RC_TAB, nel * RC_TAB * RC_Q, &T4));
  RET(wsT(S_RC_D, nel * RC_Q, &D4));
  RET(wsT(S_RC_PINF, nel, &pinf));
  RET(wsT(S_RC_DEN, 2 * nel, &den));
  dinv = den + nel;
  // share subsets per (component, block): the blocks' 4 U one-wave workgroups alone leave the chip idle when U is small
  // (the live round: one block, ~430 dependent point operations in one lane, 7 ms); each subset runs the doubling
  // chain again, so only while 4 U nsplit stays under ~one wave per SIMD
  const uint32_t nsplit = std::max(1u, std::min({8u, t, 1024u / (4 * U)}));
  RET(wsT(S_RC_A, (size_t)4 * nsplit * Ru, &A));
  RET(launch("k_rc_digits", k_rc_digits, U * RC_BLK, RC_BLK, st, U, t, maxev, ub, ref, d_selidx, naf, ev, hdr));
  for (uint32_t l = 0; l < RC_TAB; ++l) {
    RET(launch("k_rc_tab_den", k_rc_tab_den, (uint32_t)nel, 128, st, l, R, Ru, k, t, ub, d_rst, d_sel, d_S,
               (const uint4*)T4, (const uint4*)D4, pinf, den));
    RET(batch_inv((uint32_t)nel, den, dinv, st));
    RET(launch("k_rc_tab_add", k_rc_tab_add, (uint32_t)nel, 128, st, l, R, Ru, k, t, ub, d_rst, d_sel, d_S, T4, D4,
               (const uint8_t*)pinf, (const Fp*)dinv));
  }
  RET(launch("k_rc_straus", k_rc_straus, 4 * Ru * nsplit, 64, st, R, Ru, maxev, ub, d_rst, (const uint32_t*)ev,
             (const uint32_t*)hdr, (const uint4*)T4, (const uint8_t*)pinf, A, nsplit));
  return launch("k_rc_combine", k_rc_combine, Ru, 128, st, R, Ru, ub, d_rst, (const G2JStore*)A, out, nsplit);
}

// Recover after the VerifyPartial statuses are known (d_st): per round the first t valid partials, xyCommit
// dedupe; blocks of 64 rounds that selected one index set take the per-round MSM (recover.h), the others the
// Lagrange terms lambda_j S_j and row sums; compression; results copied to the output buffers (host or device
// memory: hipMemcpyDefault).
int recover_tail(uint32_t R, uint32_t k, uint32_t t, const uint8_t* d_p, const uint8_t* d_st, const G2AStore* d_S,
                 uint8_t* out_sig96, uint8_t* round_status, uint8_t* share_status, hipStream_t st) {
  uint8_t *d_rst, *d_sst, *d_out, *d_uni;
  uint32_t *d_sel, *d_selidx, *d_ref, *d_ub = nullptr;
  G2JStore* terms;
  const uint32_t nblk = (R + RC_BLK - 1) / RC_BLK;
  RET(wsT(S_SEL, (size_t)R * t, &d_sel));
  RET(wsT(S_SELIDX, (size_t)R * t, &d_selidx));
  RET(wsT(S_RST, R, &d_rst));
  RET(wsT(S_SST, (size_t)R * k, &d_sst));
  RET(launch("k_recover_select", k_recover_select, R, 128, st, R, k, t, d_p, d_st, d_sel, d_selidx, d_rst, d_sst));
  RET(wsT(S_RC_UNI, nblk, &d_uni));
  RET(wsT(S_RC_REF, nblk, &d_ref));
  RET(launch("k_rc_blocks", k_rc_blocks, nblk * RC_BLK, 64, st, R, t, (const uint32_t*)d_selidx, (const uint8_t*)d_rst,
             d_uni, d_ref));
  // the host orders the work: which blocks are uniform (and hold an OK round) decides the launch sizes
  std::vector<uint8_t> uni(nblk);
  std::vector<uint32_t> ref(nblk);
  HIPCHK(hipMemcpyAsync(uni.data(), d_uni, nblk, hipMemcpyDeviceToHost, st));
  HIPCHK(hipMemcpyAsync(ref.data(), d_ref, 4 * (size_t)nblk, hipMemcpyDeviceToHost, st));
  HIPCHK(hipStreamSynchronize(st));
  // ub: the uniform blocks holding an OK round (the block-uniform MSM); nl: every round of the other blocks (the
  // divergent-round form); one host list, uploaded once
  std::vector<uint32_t> lists;
  for (uint32_t b = 0; b < nblk; ++b)
    if (uni[b] && ref[b] != ~0u) lists.push_back(b);
  const uint32_t U = (uint32_t)lists.size();
  for (uint32_t b = 0; b < nblk; ++b)
    if (!uni[b])
      for (uint32_t r = b * RC_BLK; r < (b + 1) * RC_BLK && r < R; ++r) lists.push_back(r);
  const uint32_t Rn = (uint32_t)lists.size() - U;
  RET(wsT(S_TERMS, R, &terms));
  if (!lists.empty()) {
    RET(wsT(S_RC_LIST, lists.size(), &d_ub));
    HIPCHK(hipMemcpyAsync(d_ub, lists.data(), 4 * lists.size(), hipMemcpyHostToDevice, st));
  }
  if (Rn) RET(recover_sac(R, k, t, Rn, d_ub + U, d_selidx, d_sel, d_rst, d_S, terms, st));
  if (U) RET(recover_msm(R, k, t, U, d_ub, d_ref, d_selidx, d_sel, d_rst, d_S, terms, st));
  RET(wsT(S_OUT0, (size_t)R * 96, &d_out));
  RET(launch("k_compress_g2", k_compress_g2, R, 128, st, R, (const G2JStore*)terms, (const uint8_t*)d_rst, d_out));
  HIPCHK(hipMemcpyAsync(out_sig96, d_out, (size_t)R * 96, hipMemcpyDefault, st));
  HIPCHK(hipMemcpyAsync(round_status, d_rst, R, hipMemcpyDefault, st));
  HIPCHK(hipMemcpyAsync(share_status, d_sst, (size_t)R * k, hipMemcpyDefault, st));
  HIPCHK(hipStreamSynchronize(st));
  if (g_ctx.timing) collect_timings();
  return 0;
}

int check_args_n(size_t n) { return n > 0x7fffffffu ? fail(DG_E_ARG, "batch too large (>= 2^31 items)") : 0; }

}  // namespace

extern "C" {

int dg_init(int device) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (g_ctx.ready && g_ctx.device == device) return 0;
  int count = 0;
  if (hipGetDeviceCount(&count) != hipSuccess || count == 0) return fail(DG_E_NODEV, "no HIP device");
  if (device < 0 || device >= count) return fail(DG_E_ARG, "device index out of range");
  hipDeviceProp_t prop;
  HIPCHK(hipGetDeviceProperties(&prop, device));
  if (std::string(prop.gcnArchName).rfind("gfx950", 0) != 0)
    return fail(DG_E_NODEV, std::string("not a gfx950 device: ") + prop.gcnArchName);
  HIPCHK(hipSetDevice(device));
  if (g_hwq_supplied && !getenv("DG_QUIET"))
    fprintf(stderr, "[drand_gpu] GPU_MAX_HW_QUEUES was unset: the library asked for %s hardware queues and plans %d "
                    "workspace sets for them; a process that started HIP before loading the library has HIP's 4 -- set "
                    "GPU_MAX_HW_QUEUES before the first HIP call (DG_QUIET=1 silences this)\n",
            kDefaultHwQueues, active_sets());
  int least_prio = 0, greatest_prio = 0;  // the tail streams take the greatest
  HIPCHK(hipDeviceGetStreamPriorityRange(&least_prio, &greatest_prio));
  // (the odd sets on low-priority streams, queues of their own: 13.1 -> 12.2 M rounds/s, dropped -- DESIGN.md §5.3)
  // (16 or 32 CUs reserved for the tail streams by CU masks, the set streams masked off them: 7.7 / 12.3 M rounds/s
  // against 12.8 M, c2_negative 2.2 / 3.4 against 3.5 M -- dropped)
  for (int i = 0; i < kSets; ++i) {
    Set& x = g_ctx.sets[i];
    if (!x.stream) HIPCHK(hipStreamCreateWithFlags(&x.stream, hipStreamNonBlocking));
    if (!x.done) HIPCHK(hipEventCreateWithFlags(&x.done, hipEventDisableTiming));
    if (!x.hop) HIPCHK(hipEventCreateWithFlags(&x.hop, hipEventDisableTiming));
  }
  // (8 or 12 tail streams, or 2-4 of 6-8 at low priority: no gain)
  if (!g_ctx.tails[0]) {
    g_ctx.ntails = env_int("DG_TAIL", 1) ? Ctx::kTails : 0;
    for (int i = 0; i < g_ctx.ntails; ++i)
      HIPCHK(hipStreamCreateWithPriority(&g_ctx.tails[i], hipStreamNonBlocking, greatest_prio));
  }
  // the tail stream of a set by its position in the rotation (set_at), so the batches of one round of concurrent heads
  // -- consecutive positions -- end on different tail streams: with set i -> tail i mod 4 and the zigzag order, sets 3
  // and 7 (and 0 and 4) shared a tail stream within a round, and the second's tail waited ~12 ms for the first's
  for (int k = 0; k < kSets; ++k) {
    const int i = k < active_sets() ? set_at(k) : k;
    g_ctx.sets[i].tail_idx = g_ctx.ntails ? k % g_ctx.ntails : -1;
    g_ctx.sets[i].tail = g_ctx.ntails ? g_ctx.tails[k % g_ctx.ntails] : nullptr;
  }
  if (!g_ctx.fb_stream) HIPCHK(hipStreamCreateWithFlags(&g_ctx.fb_stream, hipStreamNonBlocking));
  // the keyed batches' side stream: a high-priority stream like the tails (a queue of its own beside the 4 normal ones,
  // so its fork / join waits stall no set stream), created here rather than on the first keyed batch
  if (!g_ctx.kc_stream) {
    HIPCHK(hipStreamCreateWithPriority(&g_ctx.kc_stream, hipStreamNonBlocking, greatest_prio));
    HIPCHK(hipEventCreateWithFlags(&g_ctx.kc_fork, hipEventDisableTiming));
    HIPCHK(hipEventCreateWithFlags(&g_ctx.kc_join, hipEventDisableTiming));
  }
  if (!g_ctx.fallbacks) {
    HIPCHK(hipMalloc(&g_ctx.fallbacks, sizeof(unsigned long long)));
    HIPCHK(hipMemset(g_ctx.fallbacks, 0, sizeof(unsigned long long)));
  }
  if (!g_ctx.gcount) {
    HIPCHK(hipMalloc(&g_ctx.gcount, GRP * sizeof(unsigned long long)));
    HIPCHK(hipMemset(g_ctx.gcount, 0, GRP * sizeof(unsigned long long)));
  }
  if (!g_ctx.xrcount) {
    HIPCHK(hipMalloc(&g_ctx.xrcount, 4 * sizeof(unsigned long long)));  // (4 words: also the prewarm's zero counters)
    HIPCHK(hipMemset(g_ctx.xrcount, 0, 4 * sizeof(unsigned long long)));
  }
  // A hardware queue's scratch (private segment) grows on the first dispatch that needs more.  On MI355X that growth,
  // when it first happened inside an overlapped batch (the round-1 per-item kernels: ~14 KB per lane), stalled every
  // queue for ~0.5 s (rocprofv3 trace), and a dispatch needing more than the queue's current segment right behind
  // another failed with HSA_STATUS_ERROR_OUT_OF_RESOURCES on the box.  So every kernel that may run on a stream is
  // dispatched there once now with no work, largest private segment first (read from the code object): the queue's
  // scratch has its final size before any batch runs.  Each queue reserves its scratch for every wave the device can
  // hold, so the two fixture kernels with the library's largest segments (k_sign, k_hash_to_g2: ~5.4 KB) have the
  // fb stream to themselves and the workspace queues hold the check pipeline's (tests/test_abi.py checks the split
  // against the code-object metadata).  With no work every lane returns at once (zero counters: xrcount).
  {
    uint32_t* z = (uint32_t*)g_ctx.xrcount;
    const uint32_t* cz = z;
    struct Warm {
      const void* fn;
      std::function<void(hipStream_t)> go;
    };
    const dim3 g1(1), b64(64), b128(128);
    const std::vector<Warm> on_sets = {
        {(const void*)k_rc_combine, [&](hipStream_t q) { hipLaunchKernelGGL(k_rc_combine, g1, b128, 0, q, 0u, 0u, (const uint32_t*)nullptr, (const uint8_t*)nullptr, (const G2JStore*)nullptr, (G2JStore*)nullptr, 1u); }},
        {(const void*)k_ck_prep, [&](hipStream_t q) { hipLaunchKernelGGL(k_ck_prep, g1, b64, 0, q, 0u, 0u, cz, 1u, (const uint64_t*)nullptr, (const G1AStore*)nullptr, cz, (const uint8_t*)nullptr, (const G2AStore*)nullptr, (uint8_t*)nullptr, (uint8_t*)nullptr, 0u, g_ctx.gcount, (CkState*)nullptr, (uint8_t*)nullptr, (RsDigits*)nullptr); }},
        {(const void*)k_ck_round_lines, [&](hipStream_t q) { hipLaunchKernelGGL(k_ck_round_lines, g1, b64, 0, q, 0u, (const G2JStore*)nullptr, (CkLine*)nullptr, (uint8_t*)nullptr); }},
        {(const void*)k_ck_lines2, [&](hipStream_t q) { hipLaunchKernelGGL(k_ck_lines2, g1, b64, 0, q, 0u, cz, (const CkState*)nullptr, (CkLine*)nullptr); }},
        {(const void*)k_ck_miller, [&](hipStream_t q) { hipLaunchKernelGGL(k_ck_miller, g1, b64, 0, q, 0u, cz, 0u, (const CkState*)nullptr, (const CkLine*)nullptr, (const CkLine*)nullptr, (Fp12*)nullptr); }},
        {(const void*)k_ck_easy, [&](hipStream_t q) { hipLaunchKernelGGL(k_ck_easy, g1, b64, 0, q, 0u, cz, 0u, (const Fp12*)nullptr, (Fp12*)nullptr, (uint32_t*)nullptr); }},
        {(const void*)k_xg_miller, [&](hipStream_t q) { hipLaunchKernelGGL(k_xg_miller, g1, b64, 0, q, 0u, cz, (const G2JStore*)nullptr, (const CkState*)nullptr, (Fp12*)nullptr); }},
        {(const void*)k_xg_heff, [&](hipStream_t q) { hipLaunchKernelGGL(k_xg_heff, g1, b64, 0, q, 0u, cz, (G2JStore*)nullptr, (CkState*)nullptr); }},
        {(const void*)k_ck_expsq2, [&](hipStream_t q) { hipLaunchKernelGGL(k_ck_expsq2, g1, b64, 0, q, 0u, cz, (const Fp12*)nullptr, (CycC*)nullptr, (Fp*)nullptr, (uint8_t*)nullptr, (uint32_t*)nullptr); }},
        {(const void*)k_ck_expdec, [&](hipStream_t q) { hipLaunchKernelGGL(k_ck_expdec, g1, b64, 0, q, 0u, cz, (const CycC*)nullptr, (Fp*)nullptr, (const uint8_t*)nullptr, (const Fp12*)nullptr, 0u, 0u, (Fp12*)nullptr); }},
        {(const void*)k_ck_explain, [&](hipStream_t q) { hipLaunchKernelGGL(k_ck_explain, g1, b64, 0, q, cz, (const Fp12*)nullptr, (const Fp12*)nullptr, 0u, 0u, (Fp12*)nullptr); }},
        {(const void*)k_ck_final, [&](hipStream_t q) { hipLaunchKernelGGL(k_ck_final, g1, b64, 0, q, 0u, cz, (const CkState*)nullptr, (const Fp12*)nullptr, (const Fp12*)nullptr, (const Fp12*)nullptr, (uint8_t*)nullptr); }},
        {(const void*)k_ck_sub, [&](hipStream_t q) { hipLaunchKernelGGL(k_ck_sub, g1, b64, 0, q, 0u, 0u, cz, (const G2AStore*)nullptr, (uint8_t*)nullptr, (uint8_t*)nullptr); }},
        {(const void*)k_ck_sac, [&](hipStream_t q) { hipLaunchKernelGGL(k_ck_sac, g1, b64, 0, q, 0u, (const uint8_t*)nullptr, (const RsDigits*)nullptr, (const uint4*)nullptr, (const uint8_t*)nullptr, (G2JStore*)nullptr, (Fp*)nullptr); }},
        {(const void*)k_xg_sub, [&](hipStream_t q) { hipLaunchKernelGGL(k_xg_sub, g1, b64, 0, q, 0u, 0u, cz, (const G2AStore*)nullptr, (uint8_t*)nullptr, z); }},
        {(const void*)k_xq_sum, [&](hipStream_t q) { hipLaunchKernelGGL(k_xq_sum, g1, b64, 0, q, 0u, 1u, (const uint64_t*)nullptr, z, cz, (const G2JStore*)nullptr, (const G2AStore*)nullptr, (uint4*)nullptr, (uint8_t*)nullptr, (G2JStore*)nullptr); }},
        {(const void*)k_xg_prep, [&](hipStream_t q) { hipLaunchKernelGGL(k_xg_prep, g1, b64, 0, q, 1u, 0u, cz, cz, 1u, cz, (const G2JStore*)nullptr, (const G2JStore*)nullptr, (const G2AStore*)nullptr, (const G1AStore*)nullptr, (CkState*)nullptr, (G2JStore*)nullptr); }},
    };
    const std::vector<Warm> on_fb = {
        {(const void*)k_sign, [&](hipStream_t q) { hipLaunchKernelGGL(k_sign, g1, b128, 0, q, 0u, (const uint8_t*)nullptr, (const uint16_t*)nullptr, (const uint8_t*)nullptr, 0u, (const uint8_t*)nullptr, 0u, (uint8_t*)nullptr); }},
        {(const void*)k_hash_to_g2, [&](hipStream_t q) { hipLaunchKernelGGL(k_hash_to_g2, g1, b128, 0, q, 0u, (const uint8_t*)nullptr, 0u, (const uint8_t*)nullptr, 0u, (uint8_t*)nullptr); }},
    };
    // largest private segment first
    auto order = [&](const std::vector<Warm>& ws, std::vector<size_t>& idx) -> int {
      std::vector<size_t> sz(ws.size());
      for (size_t i = 0; i < ws.size(); ++i) {
        hipFuncAttributes fa{};
        HIPCHK(hipFuncGetAttributes(&fa, ws[i].fn));
        sz[i] = fa.localSizeBytes;
        idx.push_back(i);
      }
      std::stable_sort(idx.begin(), idx.end(), [&](size_t a, size_t b) { return sz[a] > sz[b]; });
      return 0;
    };
    std::vector<size_t> oset, ofb;
    RET(order(on_sets, oset));
    RET(order(on_fb, ofb));
    // only the active sets' streams are dispatched to (a stream takes a hardware queue at its first dispatch), the fb
    // stream after them
    for (int i = 0; i < active_sets(); ++i)
      for (size_t w : oset) on_sets[w].go(g_ctx.sets[i].stream);
    for (size_t w : ofb) on_fb[w].go(g_ctx.fb_stream);
    for (hipStream_t t : g_ctx.tails)  // the tail streams' queues (high priority) run the check pipeline too
      if (t)
        for (size_t w : oset) on_sets[w].go(t);
  }
  HIPCHK(hipGetLastError());
  HIPCHK(hipDeviceSynchronize());
  g_ctx.device = device;
  g_ctx.ready = true;
  return 0;
}

void dg_shutdown(void) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (!g_ctx.ready) return;
  for (Set& x : g_ctx.sets) {
    if (x.stream) (void)hipStreamSynchronize(x.stream);
    for (void* p : x.pool)
      if (p) (void)hipFree(p);
    x.pool.clear();
    x.pool_size.clear();
    x.busy = false;
    if (x.stream) (void)hipStreamDestroy(x.stream);
    if (x.done) (void)hipEventDestroy(x.done);
    if (x.hop) (void)hipEventDestroy(x.hop);
    x.stream = nullptr;
    x.done = nullptr;
    x.hop = nullptr;
    x.tail = nullptr;
  }
  for (hipStream_t& t : g_ctx.tails) {
    if (t) {
      (void)hipStreamSynchronize(t);
      (void)hipStreamDestroy(t);
    }
    t = nullptr;
  }
  for (Set& x : g_ctx.xr_pools) {
    for (void* p : x.pool)
      if (p) (void)hipFree(p);
    x.pool.clear();
    x.pool_size.clear();
  }
  g_ctx.ntails = 0;
  if (g_ctx.fb_stream) {
    (void)hipStreamSynchronize(g_ctx.fb_stream);
    (void)hipStreamDestroy(g_ctx.fb_stream);
    g_ctx.fb_stream = nullptr;
  }
  if (g_ctx.kc_stream) {
    (void)hipStreamSynchronize(g_ctx.kc_stream);
    (void)hipStreamDestroy(g_ctx.kc_stream);
    (void)hipEventDestroy(g_ctx.kc_fork);
    (void)hipEventDestroy(g_ctx.kc_join);
    g_ctx.kc_stream = nullptr;
    g_ctx.kc_fork = g_ctx.kc_join = nullptr;
  }
  if (g_ctx.pk_dev) (void)hipFree(g_ctx.pk_dev);
  if (g_ctx.pk_status) (void)hipFree(g_ctx.pk_status);
  if (g_ctx.pk_raw) (void)hipFree(g_ctx.pk_raw);
  if (g_ctx.pk_ready) (void)hipEventDestroy(g_ctx.pk_ready);
  if (g_ctx.fallbacks) (void)hipFree(g_ctx.fallbacks);
  if (g_ctx.gcount) (void)hipFree(g_ctx.gcount);
  if (g_ctx.xrcount) (void)hipFree(g_ctx.xrcount);
  g_ctx.xrcount = nullptr;
  if (g_ctx.d_dst) (void)hipFree(g_ctx.d_dst);
  if (g_ctx.d_xmd) (void)hipFree(g_ctx.d_xmd);
  g_ctx.d_dst = nullptr;
  g_ctx.d_xmd = nullptr;
  g_ctx.dst_dev_valid = false;
  g_ctx.fallbacks = nullptr;
  g_ctx.gcount = nullptr;
  if (g_ctx.poly_keys) (void)hipFree(g_ctx.poly_keys);
  if (g_ctx.poly_kst) (void)hipFree(g_ctx.poly_kst);
  if (g_ctx.poly_ready) (void)hipEventDestroy(g_ctx.poly_ready);
  g_ctx.poly_keys = nullptr;
  g_ctx.poly_kst = nullptr;
  g_ctx.poly_ready = nullptr;
  g_ctx.poly_cap = 0;
  g_ctx.poly_valid = false;
  g_ctx.pk_dev = nullptr;
  g_ctx.pk_status = nullptr;
  g_ctx.pk_raw = nullptr;
  g_ctx.pk_ready = nullptr;
  g_ctx.pk_valid = false;
  g_ctx.ready = false;
}

const char* dg_last_error(void) { return g_err.c_str(); }

int dg_set_hash_dst(const uint8_t* dst, size_t dst_len) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (dst_len > 255 || (dst_len > 0 && !dst)) return fail(DG_E_ARG, "DST longer than 255 bytes");
  // batches in flight hash with the DST they were enqueued with (uploaded into their own workspace set)
  if (dst_len == 0)
    g_ctx.dst.assign(kDstNul, kDstNul + kDstNulLen);
  else
    g_ctx.dst.assign(dst, dst + dst_len);
  g_ctx.dst_dev_valid = false;
  return 0;
}

int dg_get_hash_dst(uint8_t* out, size_t cap, size_t* len) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (!len) return fail(DG_E_ARG, "bad arguments");
  *len = g_ctx.dst.size();
  if (out && cap) memcpy(out, g_ctx.dst.data(), cap < g_ctx.dst.size() ? cap : g_ctx.dst.size());
  return 0;
}

int dg_device_ready(void) { return g_ctx.ready ? 1 : 0; }

int dg_set_timing(int on) {
  std::lock_guard<std::mutex> lk(g_mu);
  g_ctx.timing = on != 0;
  g_ctx.timings.clear();
  return 0;
}

int dg_last_timings(const char** names, double* us, int* launches, int cap) {
  std::lock_guard<std::mutex> lk(g_mu);
  int k = 0;
  for (auto& t : g_ctx.timings) {
    if (k >= cap) break;
    names[k] = t.name;
    us[k] = t.launches ? t.total_us / t.launches : 0.0;
    launches[k] = t.launches;
    ++k;
  }
  return k;
}

int dg_hash_to_g2(size_t n, const uint8_t* msgs, size_t msg_len, const uint8_t* dst, size_t dst_len, uint8_t* out96) {
  std::lock_guard<std::mutex> lk(g_mu);
  RET(require_ready());
  if (n == 0) return 0;
  if (!msgs || !dst || !out96 || dst_len > 255 || n > 0xffffffffu) return fail(DG_E_ARG, "bad arguments");
  hipStream_t st;
  RET(acquire_set(&st));
  st = g_ctx.fb_stream;  // (its private segment: the per-item stream's queue holds the large scratch reservations)
  const uint8_t *d_msgs, *d_dst;
  RET(upload(S_MSGS, msgs, n * msg_len, (uint8_t**)&d_msgs, st));
  RET(upload(S_DST, dst, dst_len, (uint8_t**)&d_dst, st));
  void* p_out;
  RET(ws(S_OUT0, 96 * n, &p_out));
  RET(launch("k_hash_to_g2", k_hash_to_g2, (uint32_t)n, 128, st, (uint32_t)n, d_msgs, (uint32_t)msg_len, d_dst,
             (uint32_t)dst_len, (uint8_t*)p_out));
  HIPCHK(hipMemcpyAsync(out96, p_out, 96 * n, hipMemcpyDeviceToHost, st));
  HIPCHK(hipStreamSynchronize(st));
  if (g_ctx.timing) collect_timings();
  return 0;
}

int dg_sign(size_t n, const uint8_t* scalars32, const uint16_t* index, const uint8_t* msgs, size_t msg_len,
            uint8_t* out) {
  std::lock_guard<std::mutex> lk(g_mu);
  RET(require_ready());
  if (n == 0) return 0;
  if (!scalars32 || !msgs || !out) return fail(DG_E_ARG, "bad arguments");
  RET(check_args_n(n));
  hipStream_t st;
  RET(acquire_set(&st));
  st = g_ctx.fb_stream;  // (its private segment: the per-item stream's queue holds the large scratch reservations)
  uint8_t *d_sc, *d_m, *d_dst, *d_out;
  uint16_t* d_idx = nullptr;
  RET(upload(S_IN0, scalars32, n * 32, &d_sc, st));
  RET(upload(S_MSGS, msgs, n * msg_len, &d_m, st));
  RET(ensure_dst());
  d_dst = g_ctx.d_dst;
  if (index) RET(upload(S_IN1, index, n, &d_idx, st));
  size_t rec = index ? 98 : 96;
  RET(wsT(S_OUT0, n * rec, &d_out));
  RET(launch("k_sign", k_sign, (uint32_t)n, 128, st, (uint32_t)n, (const uint8_t*)d_sc, (const uint16_t*)d_idx,
             (const uint8_t*)d_m, (uint32_t)msg_len, (const uint8_t*)d_dst, (uint32_t)g_ctx.dst.size(), d_out));
  HIPCHK(hipMemcpyAsync(out, d_out, n * rec, hipMemcpyDeviceToHost, st));
  HIPCHK(hipStreamSynchronize(st));
  if (g_ctx.timing) collect_timings();
  return 0;
}

int dg_verify(const uint8_t pk48[48], size_t n, const uint8_t* msgs, size_t msg_len, const uint8_t* sigs96,
              uint8_t* status, uint64_t seed) {
  std::lock_guard<std::mutex> lk(g_mu);
  RET(require_ready());
  if (n == 0) return 0;
  if (!pk48 || !msgs || !sigs96 || !status) return fail(DG_E_ARG, "bad arguments");
  RET(check_args_n(n));
  hipStream_t st;
  RET(acquire_set(&st));
  uint8_t *d_msgs, *d_sigs, *d_st;
  RET(upload(S_MSGS, msgs, n * msg_len, &d_msgs, st));
  RET(upload(S_IN0, sigs96, n * 96, &d_sigs, st));
  RET(wsT(S_STATUS, n, &d_st));
  RET(verify_single_key(pk48, (uint32_t)n, d_msgs, (uint32_t)msg_len, d_sigs, d_st, fresh_seed(seed), st));
  HIPCHK(hipMemcpyAsync(status, d_st, n, hipMemcpyDeviceToHost, st));
  HIPCHK(hipStreamSynchronize(st));
  if (g_ctx.timing) collect_timings();
  return 0;
}

static int beacons_to_msgs(size_t n, const uint64_t* d_pr, const uint64_t* d_r, const uint8_t* d_ps,
                           const uint32_t* d_off, uint8_t** d_msgs, hipStream_t st) {
  RET(wsT(S_MSGS, 32 * n, d_msgs));
  return launch("k_beacon_msgs", k_beacon_msgs, (uint32_t)n, 256, st, (uint32_t)n, d_pr, d_r, d_ps, d_off, *d_msgs);
}

static int upload_beacons(size_t n, const uint64_t* prev_round, const uint64_t* round, const uint8_t* prev_sigs,
                          const uint32_t* prev_sig_off, hipStream_t st, uint64_t** d_pr, uint64_t** d_r,
                          uint8_t** d_ps, uint32_t** d_off) {
  RET(upload(S_IN1, prev_round, n, d_pr, st));
  RET(upload(S_IN2, round, n, d_r, st));
  RET(upload(S_IN3, prev_sig_off, n + 1, d_off, st));
  RET(upload(S_IN4, prev_sigs, prev_sig_off[n], d_ps, st));
  return 0;
}

// Enqueue one device-resident beacon batch on the next workspace set without waiting for it.
static int enqueue_beacons_dev(const uint8_t* pk48_host, size_t n, const uint64_t* d_pr, const uint64_t* d_r,
                               const uint8_t* d_ps, const uint32_t* d_off, const uint8_t* d_sigs, uint8_t* d_status,
                               uint64_t seed, hipStream_t in_stream, hipStream_t done_stream) {
  hipStream_t st;
  RET(acquire_set(&st));
  Set& set = cur_set();
  if (in_stream) {
    HIPCHK(hipEventRecord(set.done, in_stream));  // inputs ready
    HIPCHK(hipStreamWaitEvent(st, set.done, 0));
  }
  uint8_t* d_msgs;
  if (g_bt.on) {
    g_bt.v.push_back(BatchTrace{g_ctx.cur, bt_event(st), nullptr, nullptr});
    g_bt.cur = &g_bt.v.back();
  }
  RET(beacons_to_msgs(n, d_pr, d_r, d_ps, d_off, &d_msgs, st));
  RET(verify_single_key(pk48_host, (uint32_t)n, d_msgs, 32, d_sigs, d_status, fresh_seed(seed), st, set.tail));
  if (set.tail) st = set.tail;  // the batch ends on its tail stream
  if (g_bt.cur) {
    g_bt.cur->d = bt_event(st);
    g_bt.cur = nullptr;
  }
  HIPCHK(hipEventRecord(set.done, st));
  set.busy = true;
  g_ctx.last_stream = st;
  if (done_stream) HIPCHK(hipStreamWaitEvent(done_stream, set.done, 0));
  return 0;
}

static int wait_all() {
  if (g_hp.on) {
    fprintf(stderr, "[dg hostprof] launches %llu: %.1f us each, %.1f ms total; set waits %llu: %.1f ms total\n",
            (unsigned long long)g_hp.launches, g_hp.launches ? g_hp.launch_us / g_hp.launches : 0.0, g_hp.launch_us / 1e3,
            (unsigned long long)g_hp.waits, g_hp.wait_us / 1e3);
    g_hp = HostProf{};
    g_hp.on = true;
  }
  for (Set& x : g_ctx.sets)
    if (x.busy) {
      HIPCHK(hipEventSynchronize(x.done));
      x.busy = false;
    }
  if (g_ctx.timing) collect_timings();
  if (!g_bt.v.empty()) {
    HIPCHK(hipDeviceSynchronize());
    fprintf(stderr, "[dg batch trace] set start hop done (ms from the first start)\n");
    for (BatchTrace& b : g_bt.v) {
      float ts = 0, th = 0, td = 0;
      (void)hipEventElapsedTime(&ts, g_bt.v[0].s, b.s);
      if (b.h) (void)hipEventElapsedTime(&th, g_bt.v[0].s, b.h);
      (void)hipEventElapsedTime(&td, g_bt.v[0].s, b.d);
      fprintf(stderr, "[dg batch trace] %d %.3f %.3f %.3f\n", b.set, ts, th, td);
    }
    for (BatchTrace& b : g_bt.v)  // (after the loop: the first start is every line's reference)
      for (hipEvent_t e : {b.s, b.h, b.d})
        if (e) (void)hipEventDestroy(e);
    g_bt.v.clear();
  }
  return 0;
}

int dg_verify_beacons(const uint8_t pk48[48], size_t n, const uint64_t* prev_round, const uint64_t* round,
                      const uint8_t* prev_sigs, const uint32_t* prev_sig_off, const uint8_t* sigs96, uint8_t* status,
                      uint64_t seed) {
  std::lock_guard<std::mutex> lk(g_mu);
  RET(require_ready());
  if (n == 0) return 0;
  if (!pk48 || !prev_round || !round || !prev_sigs || !prev_sig_off || !sigs96 || !status)
    return fail(DG_E_ARG, "bad arguments");
  RET(check_args_n(n));
  hipStream_t st;
  RET(acquire_set(&st));
  uint64_t *d_pr, *d_r;
  uint8_t *d_ps, *d_sigs, *d_msgs, *d_st;
  uint32_t* d_off;
  RET(upload(S_IN0, sigs96, n * 96, &d_sigs, st));
  RET(upload_beacons(n, prev_round, round, prev_sigs, prev_sig_off, st, &d_pr, &d_r, &d_ps, &d_off));
  RET(beacons_to_msgs(n, d_pr, d_r, d_ps, d_off, &d_msgs, st));
  RET(wsT(S_STATUS, n, &d_st));
  RET(verify_single_key(pk48, (uint32_t)n, d_msgs, 32, d_sigs, d_st, fresh_seed(seed), st));
  HIPCHK(hipMemcpyAsync(status, d_st, n, hipMemcpyDeviceToHost, st));
  HIPCHK(hipStreamSynchronize(st));
  if (g_ctx.timing) collect_timings();
  return 0;
}

int dg_verify_beacons_dev(const uint8_t* pk48_host, size_t n, const uint64_t* d_prev_round, const uint64_t* d_round,
                          const uint8_t* d_prev_sigs, const uint32_t* d_prev_sig_off, const uint8_t* d_sigs96,
                          uint8_t* d_status, uint64_t seed, void* stream) {
  std::lock_guard<std::mutex> lk(g_mu);
  RET(require_ready());
  if (n == 0) return 0;
  if (!pk48_host || !d_prev_round || !d_round || !d_prev_sigs || !d_prev_sig_off || !d_sigs96 || !d_status)
    return fail(DG_E_ARG, "bad arguments");
  RET(check_args_n(n));
  RET(enqueue_beacons_dev(pk48_host, n, d_prev_round, d_round, d_prev_sigs, d_prev_sig_off, d_sigs96, d_status, seed,
                          (hipStream_t)stream, nullptr));
  RET(wait_all());
  return 0;
}

int dg_verify_beacons_dev_async(const uint8_t* pk48_host, size_t n, const uint64_t* d_prev_round,
                                const uint64_t* d_round, const uint8_t* d_prev_sigs, const uint32_t* d_prev_sig_off,
                                const uint8_t* d_sigs96, uint8_t* d_status, uint64_t seed, void* in_stream,
                                void* done_stream) {
  std::lock_guard<std::mutex> lk(g_mu);
  RET(require_ready());
  if (n == 0) return 0;
  if (!pk48_host || !d_prev_round || !d_round || !d_prev_sigs || !d_prev_sig_off || !d_sigs96 || !d_status)
    return fail(DG_E_ARG, "bad arguments");
  RET(check_args_n(n));
  return enqueue_beacons_dev(pk48_host, n, d_prev_round, d_round, d_prev_sigs, d_prev_sig_off, d_sigs96, d_status, seed,
                             (hipStream_t)in_stream, (hipStream_t)done_stream);
}

int dg_queue_plan(int hw_queues, int* sets, int* per_item_on_set_streams) {
  if (!sets || !per_item_on_set_streams) return fail(DG_E_ARG, "bad arguments");
  queue_plan(hw_queues, sets, per_item_on_set_streams);
  return 0;
}

int dg_last_batch_stream(void** out) {
  std::lock_guard<std::mutex> lk(g_mu);
  RET(require_ready());
  if (!out) return fail(DG_E_ARG, "bad arguments");
  if (!g_ctx.last_stream) return fail(DG_E_ARG, "no asynchronous batch enqueued yet");
  *out = (void*)g_ctx.last_stream;
  return 0;
}

int dg_last_batch_flags(uint32_t* out2) {
  std::lock_guard<std::mutex> lk(g_mu);
  RET(require_ready());
  RET(wait_all());
  Set& set = cur_set();
  if (set.pool.size() < S_COUNT || !set.pool[S_FLAG]) return fail(DG_E_ARG, "no batch has run");
  HIPCHK(hipMemcpy(out2, set.pool[S_FLAG], 8, hipMemcpyDeviceToHost));
  return 0;
}

int dg_fallback_count(uint64_t* out) {
  std::lock_guard<std::mutex> lk(g_mu);
  RET(require_ready());
  if (!out) return fail(DG_E_ARG, "bad arguments");
  RET(wait_all());
  unsigned long long v = 0;
  HIPCHK(hipMemcpy(&v, g_ctx.fallbacks, sizeof(v), hipMemcpyDeviceToHost));
  *out = v;
  return 0;
}

int dg_group_counts(uint64_t* out4) {
  std::lock_guard<std::mutex> lk(g_mu);
  RET(require_ready());
  if (!out4) return fail(DG_E_ARG, "bad arguments");
  RET(wait_all());
  unsigned long long v[GRP];
  HIPCHK(hipMemcpy(v, g_ctx.gcount, sizeof(v), hipMemcpyDeviceToHost));
  for (uint32_t m = 0; m < GRP; ++m) out4[m] = v[m];
  return 0;
}

int dg_isolation_counts(uint64_t* out3) {
  std::lock_guard<std::mutex> lk(g_mu);
  RET(require_ready());
  if (!out3) return fail(DG_E_ARG, "bad arguments");
  RET(wait_all());
  unsigned long long v[3];
  HIPCHK(hipMemcpy(v, g_ctx.xrcount, sizeof(v), hipMemcpyDeviceToHost));
  for (int m = 0; m < 3; ++m) out3[m] = v[m];
  return 0;
}

int dg_set_group_size(uint32_t m) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (m < 1 || m > GRP) return fail(DG_E_ARG, "group size must be 1..4");
  g_group_size = m;
  return 0;
}

int dg_wait_all(void) {
  std::lock_guard<std::mutex> lk(g_mu);
  RET(require_ready());
  return wait_all();
}

int dg_check_links(uint64_t cur_round, const uint8_t* cur_sig, size_t cur_sig_len, size_t n, const uint64_t* prev_round,
                   const uint64_t* round, const uint8_t* prev_sigs, const uint32_t* prev_sig_off, const uint8_t* sigs96,
                   uint8_t* link_status) {
  std::lock_guard<std::mutex> lk(g_mu);
  RET(require_ready());
  if (n == 0) return 0;
  if (!cur_sig || !prev_round || !round || !prev_sigs || !prev_sig_off || !sigs96 || !link_status)
    return fail(DG_E_ARG, "bad arguments");
  RET(check_args_n(n));
  hipStream_t st;
  RET(acquire_set(&st));
  uint64_t *d_pr, *d_r;
  uint8_t *d_ps, *d_sigs, *d_cur, *d_out;
  uint32_t* d_off;
  RET(upload(S_IN0, sigs96, n * 96, &d_sigs, st));
  RET(upload_beacons(n, prev_round, round, prev_sigs, prev_sig_off, st, &d_pr, &d_r, &d_ps, &d_off));
  RET(upload(S_DST, cur_sig, cur_sig_len, &d_cur, st));
  RET(wsT(S_OUT0, n, &d_out));
  RET(launch("k_links", k_links, (uint32_t)n, 256, st, (uint32_t)n, cur_round, (const uint8_t*)d_cur,
             (uint32_t)cur_sig_len, (const uint64_t*)d_pr, (const uint64_t*)d_r, (const uint8_t*)d_ps,
             (const uint32_t*)d_off, (const uint8_t*)d_sigs, d_out));
  HIPCHK(hipMemcpyAsync(link_status, d_out, n, hipMemcpyDeviceToHost, st));
  HIPCHK(hipStreamSynchronize(st));
  return 0;
}

int dg_beacon_messages(size_t n, const uint64_t* prev_round, const uint64_t* round, const uint8_t* prev_sigs,
                       const uint32_t* prev_sig_off, uint8_t* out32) {
  std::lock_guard<std::mutex> lk(g_mu);
  RET(require_ready());
  if (n == 0) return 0;
  if (!prev_round || !round || !prev_sigs || !prev_sig_off || !out32) return fail(DG_E_ARG, "bad arguments");
  RET(check_args_n(n));
  hipStream_t st;
  RET(acquire_set(&st));
  uint64_t *d_pr, *d_r;
  uint8_t *d_ps, *d_msgs;
  uint32_t* d_off;
  RET(upload_beacons(n, prev_round, round, prev_sigs, prev_sig_off, st, &d_pr, &d_r, &d_ps, &d_off));
  RET(beacons_to_msgs(n, d_pr, d_r, d_ps, d_off, &d_msgs, st));
  HIPCHK(hipMemcpyAsync(out32, d_msgs, 32 * n, hipMemcpyDeviceToHost, st));
  HIPCHK(hipStreamSynchronize(st));
  return 0;
}

int dg_randomness(size_t n, const uint8_t* sigs96, uint8_t* out32) {
  std::lock_guard<std::mutex> lk(g_mu);
  RET(require_ready());
  if (n == 0) return 0;
  if (!sigs96 || !out32) return fail(DG_E_ARG, "bad arguments");
  RET(check_args_n(n));
  hipStream_t st;
  RET(acquire_set(&st));
  uint8_t *d_sigs, *d_out;
  RET(upload(S_IN0, sigs96, n * 96, &d_sigs, st));
  RET(wsT(S_OUT0, 32 * n, &d_out));
  RET(launch("k_randomness", k_randomness, (uint32_t)n, 256, st, (uint32_t)n, (const uint8_t*)d_sigs, d_out));
  HIPCHK(hipMemcpyAsync(out32, d_out, 32 * n, hipMemcpyDeviceToHost, st));
  HIPCHK(hipStreamSynchronize(st));
  return 0;
}

int dg_pubpoly_eval(const uint8_t* commits48, uint32_t t, size_t n, const uint32_t* index, uint8_t* out48) {
  std::lock_guard<std::mutex> lk(g_mu);
  RET(require_ready());
  if (n == 0) return 0;
  if (!commits48 || t == 0 || !index || !out48) return fail(DG_E_ARG, "bad arguments");
  RET(check_args_n(n));
  hipStream_t st;
  RET(acquire_set(&st));
  uint8_t *d_c, *d_cst, *d_out, *d_kst;
  uint32_t* d_idx;
  G1AStore *cA, *keys;
  RET(upload(S_IN0, commits48, (size_t)t * 48, &d_c, st));
  RET(wsT(S_COMMITS, t, &cA));
  RET(wsT(S_COMMITST, t, &d_cst));
  RET(launch("k_decode_g1", k_decode_g1, t, 64, st, t, (const uint8_t*)d_c, cA, d_cst));
  RET(upload(S_SLOTIDX, index, n, &d_idx, st));
  RET(wsT(S_KEYS, n, &keys));
  RET(wsT(S_KEYST, n, &d_kst));
  RET(wsT(S_OUT0, 48 * n, &d_out));
  RET(launch("k_pubpoly_eval", k_pubpoly_eval, (uint32_t)n, 64, st, (uint32_t)n, t, (const G1AStore*)cA,
             (const uint8_t*)d_cst, (const uint32_t*)d_idx, keys, d_kst, d_out));
  std::vector<uint8_t> kst(n);
  HIPCHK(hipMemcpyAsync(out48, d_out, 48 * n, hipMemcpyDeviceToHost, st));
  HIPCHK(hipMemcpyAsync(kst.data(), d_kst, n, hipMemcpyDeviceToHost, st));
  HIPCHK(hipStreamSynchronize(st));
  if (g_ctx.timing) collect_timings();
  if (kst[0] != DG_ST_OK) return fail(DG_E_ARG, "a commitment does not decode");
  return 0;
}

int dg_verify_partials(const uint8_t* commits48, uint32_t t, size_t rounds, const uint8_t* msgs, size_t msg_len,
                       uint32_t k, const uint8_t* partials98, uint8_t* status, uint64_t seed) {
  std::lock_guard<std::mutex> lk(g_mu);
  RET(require_ready());
  if (rounds == 0 || k == 0) return 0;
  if (!commits48 || t == 0 || !msgs || !partials98 || !status) return fail(DG_E_ARG, "bad arguments");
  RET(check_args_n(rounds * (size_t)k));
  hipStream_t st;
  RET(acquire_set0(&st));
  uint8_t *d_st, *d_m, *d_p;
  RET(upload(S_MSGS, msgs, rounds * msg_len, &d_m, st));
  RET(upload(S_IN1, partials98, rounds * k * 98, &d_p, st));
  RET(verify_partials_dev(commits48, t, (uint32_t)rounds, d_m, (uint32_t)msg_len, k, d_p, fresh_seed(seed), st, &d_st));
  HIPCHK(hipMemcpyAsync(status, d_st, rounds * k, hipMemcpyDeviceToHost, st));
  HIPCHK(hipStreamSynchronize(st));
  if (g_ctx.timing) collect_timings();
  return 0;
}

int dg_verify_partials_dev(const uint8_t* commits48, uint32_t t, size_t rounds, const uint8_t* d_msgs, size_t msg_len,
                           uint32_t k, const uint8_t* d_partials98, uint8_t* d_status, uint64_t seed) {
  std::lock_guard<std::mutex> lk(g_mu);
  RET(require_ready());
  if (rounds == 0 || k == 0) return 0;
  if (!commits48 || t == 0 || !d_msgs || !d_partials98 || !d_status) return fail(DG_E_ARG, "bad arguments");
  RET(check_args_n(rounds * (size_t)k));
  hipStream_t st;
  RET(acquire_set0(&st));
  uint8_t* d_st;
  RET(verify_partials_dev(commits48, t, (uint32_t)rounds, d_msgs, (uint32_t)msg_len, k, d_partials98, fresh_seed(seed),
                          st, &d_st));
  HIPCHK(hipMemcpyAsync(d_status, d_st, rounds * k, hipMemcpyDeviceToDevice, st));
  HIPCHK(hipStreamSynchronize(st));
  if (g_ctx.timing) collect_timings();
  return 0;
}

int dg_recover(const uint8_t* commits48, uint32_t t, uint32_t nshares, size_t rounds, const uint8_t* msgs,
               size_t msg_len, uint32_t k, const uint8_t* partials98, uint8_t* out_sig96, uint8_t* round_status,
               uint8_t* share_status, uint64_t seed) {
  std::lock_guard<std::mutex> lk(g_mu);
  RET(require_ready());
  (void)nshares;  // kyber passes n to RecoverCommit only as a capacity hint
  if (rounds == 0) return 0;
  if (!commits48 || t == 0 || k == 0 || !msgs || !partials98 || !out_sig96 || !round_status || !share_status)
    return fail(DG_E_ARG, "bad arguments");
  RET(check_args_n(rounds * (size_t)(k > t ? k : t)));
  hipStream_t st;
  RET(acquire_set0(&st));
  const uint32_t R = (uint32_t)rounds;
  uint8_t *d_st, *d_m, *d_p;
  G2AStore* d_S;
  RET(upload(S_MSGS, msgs, (size_t)R * msg_len, &d_m, st));
  RET(upload(S_IN1, partials98, (size_t)R * k * 98, &d_p, st));
  RET(recover_windowed(commits48, t, R, d_m, (uint32_t)msg_len, k, d_p, fresh_seed(seed), st, &d_st, &d_S));
  return recover_tail(R, k, t, d_p, d_st, d_S, out_sig96, round_status, share_status, st);
}

int dg_recover_dev(const uint8_t* commits48, uint32_t t, uint32_t nshares, size_t rounds, const uint8_t* d_msgs,
                   size_t msg_len, uint32_t k, const uint8_t* d_partials98, uint8_t* d_out_sig96,
                   uint8_t* d_round_status, uint8_t* d_share_status, uint64_t seed) {
  std::lock_guard<std::mutex> lk(g_mu);
  RET(require_ready());
  (void)nshares;
  if (rounds == 0) return 0;
  if (!commits48 || t == 0 || k == 0 || !d_msgs || !d_partials98 || !d_out_sig96 || !d_round_status ||
      !d_share_status)
    return fail(DG_E_ARG, "bad arguments");
  RET(check_args_n(rounds * (size_t)(k > t ? k : t)));
  hipStream_t st;
  RET(acquire_set0(&st));
  const uint32_t R = (uint32_t)rounds;
  uint8_t* d_st;
  G2AStore* d_S;
  RET(recover_windowed(commits48, t, R, d_msgs, (uint32_t)msg_len, k, d_partials98, fresh_seed(seed), st, &d_st, &d_S));
  return recover_tail(R, k, t, d_partials98, d_st, d_S, d_out_sig96, d_round_status, d_share_status, st);
}

// sigma of every partial decoded by the phase kernels, then the known verdicts carried over (k_merge_verified)
static int decode_verified(uint32_t N, const uint8_t* d_p, const uint8_t* d_vst, G2AStore* d_S, uint8_t* d_st,
                           hipStream_t st) {
  uint8_t *kok, *iso;
  RET(wsT(S_KOK, 16, &kok));
  RET(wsT(S_ISO, N, &iso));
  HIPCHK(hipMemsetAsync(kok, 0, 16, st));  // one "key" with an OK status: no key side on this path
  RET(decode_items(N, 1, 0, d_p, 98, 2, nullptr, kok, d_S, d_st, nullptr, iso, 0u, st));
  return launch("k_merge_verified", k_merge_verified, N, 128, st, N, d_vst, d_S, d_st);
}

int dg_recover_verified(uint32_t t, uint32_t nshares, size_t rounds, uint32_t k, const uint8_t* partials98,
                        const uint8_t* verified_status, uint8_t* out_sig96, uint8_t* round_status,
                        uint8_t* share_status) {
  std::lock_guard<std::mutex> lk(g_mu);
  RET(require_ready());
  (void)nshares;
  if (rounds == 0) return 0;
  if (t == 0 || k == 0 || !partials98 || !verified_status || !out_sig96 || !round_status || !share_status)
    return fail(DG_E_ARG, "bad arguments");
  RET(check_args_n(rounds * (size_t)(k > t ? k : t)));
  hipStream_t st;
  RET(acquire_set0(&st));
  const uint32_t R = (uint32_t)rounds;
  const size_t N = (size_t)R * k;
  uint8_t *d_p, *d_vst, *d_st;
  G2AStore* d_S;
  RET(upload(S_IN1, partials98, N * 98, &d_p, st));
  RET(upload(S_VST, verified_status, N, &d_vst, st));
  RET(wsT(S_STATUS, N, &d_st));
  RET(wsT(S_S, N, &d_S));
  RET(decode_verified((uint32_t)N, d_p, d_vst, d_S, d_st, st));
  return recover_tail(R, k, t, d_p, d_st, d_S, out_sig96, round_status, share_status, st);
}

int dg_recover_verified_dev(uint32_t t, uint32_t nshares, size_t rounds, uint32_t k, const uint8_t* d_partials98,
                            const uint8_t* d_verified_status, uint8_t* d_out_sig96, uint8_t* d_round_status,
                            uint8_t* d_share_status) {
  std::lock_guard<std::mutex> lk(g_mu);
  RET(require_ready());
  (void)nshares;
  if (rounds == 0) return 0;
  if (t == 0 || k == 0 || !d_partials98 || !d_verified_status || !d_out_sig96 || !d_round_status || !d_share_status)
    return fail(DG_E_ARG, "bad arguments");
  RET(check_args_n(rounds * (size_t)(k > t ? k : t)));
  hipStream_t st;
  RET(acquire_set0(&st));
  const uint32_t R = (uint32_t)rounds;
  const size_t N = (size_t)R * k;
  uint8_t* d_st;
  G2AStore* d_S;
  RET(wsT(S_STATUS, N, &d_st));
  RET(wsT(S_S, N, &d_S));
  RET(decode_verified((uint32_t)N, d_partials98, d_verified_status, d_S, d_st, st));
  return recover_tail(R, k, t, d_partials98, d_st, d_S, d_out_sig96, d_round_status, d_share_status, st);
}

}  // extern "C"
