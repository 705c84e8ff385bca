// libdrandgpu.so: the C-ABI of include/drand_gpu.h over the HIP kernels of kernels.h (gfx950 only).
// Host code here only moves bytes, sizes launches and sequences kernels; every group/field operation
// runs on the device.  No CPU fallback exists: without a gfx950 device the API returns DG_E_NODEV.
#include <hip/hip_runtime.h>

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

struct Ctx {
  int device = -1;
  bool ready = false;
  hipStream_t stream = nullptr;
  std::vector<void*> pool;  // grow-only device allocations, indexed by slot
  std::vector<size_t> pool_size;
  bool timing = false;
  std::vector<Timing> timings;
  std::vector<std::pair<hipEvent_t, hipEvent_t>> pending;
  std::vector<const char*> pending_names;
  std::vector<hipEvent_t> free_events;
};

std::mutex g_mu;
Ctx g_ctx;
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
  S_MSGS, S_DST, S_Q, S_S, S_STATUS, S_R, S_T, S_SUM_A, S_SUM_B, S_PK, S_PKST, S_FLAG, S_IN0, S_IN1, S_IN2, S_IN3, S_IN4,
  S_OUT0, S_OUT1, S_COUNT
};

int ws(Slot s, size_t bytes, void** out) {
  Ctx& c = g_ctx;
  if (c.pool.size() < S_COUNT) {
    c.pool.assign(S_COUNT, nullptr);
    c.pool_size.assign(S_COUNT, 0);
  }
  if (bytes == 0) bytes = 16;
  if (c.pool_size[s] < bytes) {
    if (c.pool[s]) HIPCHK(hipFree(c.pool[s]));
    c.pool[s] = nullptr;
    size_t sz = bytes + bytes / 4;
    HIPCHK(hipMalloc(&c.pool[s], sz));
    c.pool_size[s] = sz;
  }
  *out = c.pool[s];
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
  hipEventCreate(&e);
  return e;
}

// launch helper with optional per-kernel event timing
template <typename... Args>
int launch(const char* name, void (*k)(Args...), uint32_t n_threads, uint32_t block, hipStream_t st, Args... args) {
  if (n_threads == 0) return 0;
  uint32_t grid = (n_threads + block - 1) / block;
  Ctx& c = g_ctx;
  hipEvent_t e0 = nullptr, e1 = nullptr;
  if (c.timing) {
    e0 = get_event();
    e1 = get_event();
    hipEventRecord(e0, st);
  }
  hipLaunchKernelGGL(k, dim3(grid), dim3(block), 0, st, args...);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return fail(DG_E_HIP, std::string("launch ") + name + ": " + hipGetErrorString(e));
  if (c.timing) {
    hipEventRecord(e1, st);
    c.pending.push_back({e0, e1});
    c.pending_names.push_back(name);
  }
  return 0;
}

void collect_timings() {
  Ctx& c = g_ctx;
  for (size_t i = 0; i < c.pending.size(); ++i) {
    float ms = 0;
    hipEventSynchronize(c.pending[i].second);
    hipEventElapsedTime(&ms, c.pending[i].first, c.pending[i].second);
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

// Sum n Jacobian points in `buf` (overwritten) down to one point at buf[0], using `tmp` as scratch.
int reduce_points(G2JStore* buf, G2JStore* tmp, uint32_t n, hipStream_t st) {
  const uint32_t chunk = 32;
  G2JStore* src = buf;
  G2JStore* dst = tmp;
  while (n > 1) {
    uint32_t m = (n + chunk - 1) / chunk;
    RET(launch("k_sum_points", k_sum_points, m, 128, st, n, chunk, (const G2JStore*)src, dst));
    n = m;
    G2JStore* t = src;
    src = dst;
    dst = t;
  }
  if (src != buf) HIPCHK(hipMemcpyAsync(buf, src, sizeof(G2JStore), hipMemcpyDeviceToDevice, st));
  return 0;
}

// Core of dg_verify / dg_verify_beacons on device buffers: d_msgs (n x msg_len), d_sigs96 -> d_status.
int verify_core(const uint8_t* pk48_host, size_t n, const uint8_t* d_msgs, uint32_t msg_len, const uint8_t* d_sigs96,
                uint8_t* d_status, uint64_t seed, hipStream_t st) {
  void *p_dst, *p_q, *p_s, *p_r, *p_t, *p_pk, *p_pkst, *p_flag;
  RET(ws(S_DST, 64, &p_dst));
  RET(ws(S_Q, sizeof(G2JStore) * n, &p_q));
  RET(ws(S_S, sizeof(G2AStore) * n, &p_s));
  RET(ws(S_R, sizeof(G2JStore) * n, &p_r));
  RET(ws(S_T, sizeof(G2JStore) * n, &p_t));
  RET(ws(S_PK, sizeof(G1AStore) + 48, &p_pk));
  RET(ws(S_PKST, 16, &p_pkst));
  RET(ws(S_FLAG, 16, &p_flag));
  uint8_t* dst = (uint8_t*)p_dst;
  HIPCHK(hipMemcpyAsync(dst, kDstNul, kDstNulLen, hipMemcpyHostToDevice, st));
  uint8_t* pk_raw = (uint8_t*)p_pk + sizeof(G1AStore);
  HIPCHK(hipMemcpyAsync(pk_raw, pk48_host, 48, hipMemcpyHostToDevice, st));
  G1AStore* pk = (G1AStore*)p_pk;
  RET(launch("k_decode_g1", k_decode_g1, 1, 64, st, 1u, (const uint8_t*)pk_raw, pk, (uint8_t*)p_pkst));
  uint8_t pk_status = 0;
  HIPCHK(hipMemcpyAsync(&pk_status, p_pkst, 1, hipMemcpyDeviceToHost, st));
  HIPCHK(hipStreamSynchronize(st));
  if (pk_status != DG_ST_OK) {
    HIPCHK(hipMemsetAsync(d_status, DG_ST_PK_DECODE, n, st));
    HIPCHK(hipStreamSynchronize(st));
    return 0;
  }
  uint32_t nn = (uint32_t)n;
  G2JStore* Q = (G2JStore*)p_q;
  G2AStore* S = (G2AStore*)p_s;
  RET(launch("k_h2c_uncleared", k_h2c_uncleared, nn, 128, st, nn, d_msgs, msg_len, (const uint8_t*)dst, kDstNulLen, Q));
  RET(launch("k_decode_sigs", k_decode_sigs, nn, 128, st, nn, d_sigs96, 96u, 0u, S, d_status));
  G2JStore* R = (G2JStore*)p_r;
  G2JStore* T = (G2JStore*)p_t;
  RET(launch("k_rlc_scale", k_rlc_scale, nn, 128, st, nn, seed, (const G2JStore*)Q, (const G2AStore*)S,
             (const uint8_t*)d_status, R, T));
  // reduce R and T in place (use the other's tail as scratch is unsafe: reduce separately with Q as tmp)
  RET(reduce_points(R, Q, nn, st));
  // Q has been clobbered by the reduction scratch; T reduction reuses it too
  RET(reduce_points(T, Q, nn, st));
  uint32_t* flag = (uint32_t*)p_flag;
  RET(launch("k_rlc_final", k_rlc_final, 1, 64, st, (const G1AStore*)pk, (const G2JStore*)R, (const G2JStore*)T, flag));
  uint32_t ok = 0;
  HIPCHK(hipMemcpyAsync(&ok, flag, 4, hipMemcpyDeviceToHost, st));
  HIPCHK(hipStreamSynchronize(st));
  if (!ok) {
    // isolate: per-item pairing check (recompute the hashes clobbered by the reduction)
    RET(launch("k_h2c_uncleared", k_h2c_uncleared, nn, 128, st, nn, d_msgs, msg_len, (const uint8_t*)dst, kDstNulLen,
               Q));
    RET(launch("k_verify_items", k_verify_items, nn, 64, st, nn, (const G1AStore*)pk, (const uint32_t*)nullptr,
               (const G2JStore*)Q, (const uint32_t*)nullptr, (const G2AStore*)S, d_status));
    HIPCHK(hipStreamSynchronize(st));
  }
  if (g_ctx.timing) collect_timings();
  return 0;
}

template <typename T>
int upload(Slot s, const T* host, size_t count, T** dev, hipStream_t st) {
  void* p;
  RET(ws(s, sizeof(T) * count, &p));
  if (count) HIPCHK(hipMemcpyAsync(p, host, sizeof(T) * count, hipMemcpyHostToDevice, st));
  *dev = (T*)p;
  return 0;
}

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
  if (!g_ctx.stream) HIPCHK(hipStreamCreateWithFlags(&g_ctx.stream, hipStreamNonBlocking));
  g_ctx.device = device;
  g_ctx.ready = true;
  return 0;
}

void dg_shutdown(void) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (!g_ctx.ready) return;
  for (void* p : g_ctx.pool)
    if (p) hipFree(p);
  g_ctx.pool.clear();
  g_ctx.pool_size.clear();
  if (g_ctx.stream) hipStreamDestroy(g_ctx.stream);
  g_ctx.stream = nullptr;
  g_ctx.ready = false;
}

const char* dg_last_error(void) { return g_err.c_str(); }

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
  hipStream_t st = g_ctx.stream;
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

int dg_verify(const uint8_t pk48[48], size_t n, const uint8_t* msgs, size_t msg_len, const uint8_t* sigs96,
              uint8_t* status, uint64_t seed) {
  std::lock_guard<std::mutex> lk(g_mu);
  RET(require_ready());
  if (n == 0) return 0;
  if (!pk48 || !msgs || !sigs96 || !status || n > 0xffffffffu) return fail(DG_E_ARG, "bad arguments");
  hipStream_t st = g_ctx.stream;
  uint8_t *d_msgs, *d_sigs;
  RET(upload(S_MSGS, msgs, n * msg_len, &d_msgs, st));
  RET(upload(S_IN0, sigs96, n * 96, &d_sigs, st));
  void* p_st;
  RET(ws(S_STATUS, n, &p_st));
  RET(verify_core(pk48, n, d_msgs, (uint32_t)msg_len, d_sigs, (uint8_t*)p_st, fresh_seed(seed), st));
  HIPCHK(hipMemcpyAsync(status, p_st, n, hipMemcpyDeviceToHost, st));
  HIPCHK(hipStreamSynchronize(st));
  return 0;
}

static int beacons_to_msgs(size_t n, const uint64_t* d_pr, const uint64_t* d_r, const uint8_t* d_ps,
                           const uint32_t* d_off, uint8_t** d_msgs, hipStream_t st) {
  void* p;
  RET(ws(S_MSGS, 32 * n, &p));
  RET(launch("k_beacon_msgs", k_beacon_msgs, (uint32_t)n, 256, st, (uint32_t)n, d_pr, d_r, d_ps, d_off, (uint8_t*)p));
  *d_msgs = (uint8_t*)p;
  return 0;
}

int dg_verify_beacons(const uint8_t pk48[48], size_t n, const uint64_t* prev_round, const uint64_t* round,
                      const uint8_t* prev_sigs, const uint32_t* prev_sig_off, const uint8_t* sigs96, uint8_t* status,
                      uint64_t seed) {
  std::lock_guard<std::mutex> lk(g_mu);
  RET(require_ready());
  if (n == 0) return 0;
  if (!pk48 || !prev_round || !round || !prev_sigs || !prev_sig_off || !sigs96 || !status || n > 0xffffffffu)
    return fail(DG_E_ARG, "bad arguments");
  hipStream_t st = g_ctx.stream;
  uint64_t *d_pr, *d_r;
  uint8_t *d_ps, *d_sigs, *d_msgs;
  uint32_t* d_off;
  RET(upload(S_IN0, sigs96, n * 96, &d_sigs, st));
  RET(upload(S_IN1, prev_round, n, &d_pr, st));
  RET(upload(S_IN2, round, n, &d_r, st));
  RET(upload(S_IN3, prev_sig_off, n + 1, &d_off, st));
  RET(upload(S_IN4, prev_sigs, prev_sig_off[n], &d_ps, st));
  RET(beacons_to_msgs(n, d_pr, d_r, d_ps, d_off, &d_msgs, st));
  void* p_st;
  RET(ws(S_STATUS, n, &p_st));
  RET(verify_core(pk48, n, d_msgs, 32, d_sigs, (uint8_t*)p_st, fresh_seed(seed), st));
  HIPCHK(hipMemcpyAsync(status, p_st, n, hipMemcpyDeviceToHost, st));
  HIPCHK(hipStreamSynchronize(st));
  return 0;
}

int dg_verify_beacons_dev(const uint8_t* pk48_host, size_t n, const uint64_t* d_prev_round, const uint64_t* d_round,
                          const uint8_t* d_prev_sigs, const uint32_t* d_prev_sig_off, const uint8_t* d_sigs96,
                          uint8_t* d_status, uint64_t seed, void* stream) {
  std::lock_guard<std::mutex> lk(g_mu);
  RET(require_ready());
  if (n == 0) return 0;
  hipStream_t st = stream ? (hipStream_t)stream : g_ctx.stream;
  uint8_t* d_msgs;
  RET(beacons_to_msgs(n, d_prev_round, d_round, d_prev_sigs, d_prev_sig_off, &d_msgs, st));
  RET(verify_core(pk48_host, n, d_msgs, 32, d_sigs96, d_status, fresh_seed(seed), st));
  HIPCHK(hipStreamSynchronize(st));
  return 0;
}

int dg_check_links(uint64_t cur_round, const uint8_t* cur_sig, size_t cur_sig_len, size_t n, const uint64_t* prev_round,
                   const uint64_t* round, const uint8_t* prev_sigs, const uint32_t* prev_sig_off, const uint8_t* sigs96,
                   uint8_t* link_status) {
  std::lock_guard<std::mutex> lk(g_mu);
  RET(require_ready());
  if (n == 0) return 0;
  hipStream_t st = g_ctx.stream;
  uint64_t *d_pr, *d_r;
  uint8_t *d_ps, *d_sigs, *d_cur;
  uint32_t* d_off;
  RET(upload(S_IN0, sigs96, n * 96, &d_sigs, st));
  RET(upload(S_IN1, prev_round, n, &d_pr, st));
  RET(upload(S_IN2, round, n, &d_r, st));
  RET(upload(S_IN3, prev_sig_off, n + 1, &d_off, st));
  RET(upload(S_IN4, prev_sigs, prev_sig_off[n], &d_ps, st));
  RET(upload(S_DST, cur_sig, cur_sig_len, &d_cur, st));
  void* p_out;
  RET(ws(S_OUT0, n, &p_out));
  RET(launch("k_links", k_links, (uint32_t)n, 256, st, (uint32_t)n, cur_round, (const uint8_t*)d_cur,
             (uint32_t)cur_sig_len, (const uint64_t*)d_pr, (const uint64_t*)d_r, (const uint8_t*)d_ps,
             (const uint32_t*)d_off, (const uint8_t*)d_sigs, (uint8_t*)p_out));
  HIPCHK(hipMemcpyAsync(link_status, p_out, n, hipMemcpyDeviceToHost, st));
  HIPCHK(hipStreamSynchronize(st));
  return 0;
}

int dg_beacon_messages(size_t n, const uint64_t* prev_round, const uint64_t* round, const uint8_t* prev_sigs,
                       const uint32_t* prev_sig_off, uint8_t* out32) {
  std::lock_guard<std::mutex> lk(g_mu);
  RET(require_ready());
  if (n == 0) return 0;
  hipStream_t st = g_ctx.stream;
  uint64_t *d_pr, *d_r;
  uint8_t *d_ps, *d_msgs;
  uint32_t* d_off;
  RET(upload(S_IN1, prev_round, n, &d_pr, st));
  RET(upload(S_IN2, round, n, &d_r, st));
  RET(upload(S_IN3, prev_sig_off, n + 1, &d_off, st));
  RET(upload(S_IN4, prev_sigs, prev_sig_off[n], &d_ps, st));
  RET(beacons_to_msgs(n, d_pr, d_r, d_ps, d_off, &d_msgs, st));
  HIPCHK(hipMemcpyAsync(out32, d_msgs, 32 * n, hipMemcpyDeviceToHost, st));
  HIPCHK(hipStreamSynchronize(st));
  return 0;
}

int dg_randomness(size_t n, const uint8_t* sigs96, uint8_t* out32) {
  std::lock_guard<std::mutex> lk(g_mu);
  RET(require_ready());
  if (n == 0) return 0;
  hipStream_t st = g_ctx.stream;
  uint8_t* d_sigs;
  RET(upload(S_IN0, sigs96, n * 96, &d_sigs, st));
  void* p_out;
  RET(ws(S_OUT0, 32 * n, &p_out));
  RET(launch("k_randomness", k_randomness, (uint32_t)n, 256, st, (uint32_t)n, (const uint8_t*)d_sigs, (uint8_t*)p_out));
  HIPCHK(hipMemcpyAsync(out32, p_out, 32 * n, hipMemcpyDeviceToHost, st));
  HIPCHK(hipStreamSynchronize(st));
  return 0;
}

}  // extern "C"
