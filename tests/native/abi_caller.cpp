// A C++ caller of include/drand_gpu.h, compiled against the header (not ctypes): every entry point is bound
// to a function pointer of the exact type a cgo / C client would see, so signature drift between the header
// and the library fails the build, and then called once without a device (every compute call must return
// DG_E_NODEV: there is no CPU fallback).  Built with ASan + UBSan by tests/test_abi.py.  Test tool only.
#include <stdio.h>
#include <string.h>

#include <type_traits>

#include "../../include/drand_gpu.h"

#define EXPECT_TYPE(fn, ...) static_assert(std::is_same<decltype(&fn), __VA_ARGS__>::value, #fn " signature")
EXPECT_TYPE(dg_init, int (*)(int));
EXPECT_TYPE(dg_shutdown, void (*)(void));
EXPECT_TYPE(dg_last_error, const char* (*)(void));
EXPECT_TYPE(dg_device_ready, int (*)(void));
EXPECT_TYPE(dg_set_hash_dst, int (*)(const uint8_t*, size_t));
EXPECT_TYPE(dg_get_hash_dst, int (*)(uint8_t*, size_t, size_t*));
EXPECT_TYPE(dg_hash_to_g2, int (*)(size_t, const uint8_t*, size_t, const uint8_t*, size_t, uint8_t*));
EXPECT_TYPE(dg_sign, int (*)(size_t, const uint8_t*, const uint16_t*, const uint8_t*, size_t, uint8_t*));
EXPECT_TYPE(dg_verify, int (*)(const uint8_t*, size_t, const uint8_t*, size_t, const uint8_t*, uint8_t*, uint64_t));
EXPECT_TYPE(dg_verify_beacons, int (*)(const uint8_t*, size_t, const uint64_t*, const uint64_t*, const uint8_t*,
                                       const uint32_t*, const uint8_t*, uint8_t*, uint64_t));
EXPECT_TYPE(dg_check_links, int (*)(uint64_t, const uint8_t*, size_t, size_t, const uint64_t*, const uint64_t*,
                                    const uint8_t*, const uint32_t*, const uint8_t*, uint8_t*));
EXPECT_TYPE(dg_beacon_messages, int (*)(size_t, const uint64_t*, const uint64_t*, const uint8_t*, const uint32_t*,
                                        uint8_t*));
EXPECT_TYPE(dg_randomness, int (*)(size_t, const uint8_t*, uint8_t*));
EXPECT_TYPE(dg_pubpoly_eval, int (*)(const uint8_t*, uint32_t, size_t, const uint32_t*, uint8_t*));
EXPECT_TYPE(dg_verify_partials, int (*)(const uint8_t*, uint32_t, size_t, const uint8_t*, size_t, uint32_t,
                                        const uint8_t*, uint8_t*, uint64_t));
EXPECT_TYPE(dg_recover, int (*)(const uint8_t*, uint32_t, uint32_t, size_t, const uint8_t*, size_t, uint32_t,
                                const uint8_t*, uint8_t*, uint8_t*, uint8_t*, uint64_t));
EXPECT_TYPE(dg_recover_verified, int (*)(uint32_t, uint32_t, size_t, uint32_t, const uint8_t*, const uint8_t*,
                                         uint8_t*, uint8_t*, uint8_t*));
EXPECT_TYPE(dg_verify_beacons_dev, int (*)(const uint8_t*, size_t, const uint64_t*, const uint64_t*, const uint8_t*,
                                           const uint32_t*, const uint8_t*, uint8_t*, uint64_t, void*));
EXPECT_TYPE(dg_verify_beacons_dev_async, int (*)(const uint8_t*, size_t, const uint64_t*, const uint64_t*,
                                                 const uint8_t*, const uint32_t*, const uint8_t*, uint8_t*, uint64_t,
                                                 void*, void*));
EXPECT_TYPE(dg_queue_plan, int (*)(int, int*, int*));
EXPECT_TYPE(dg_last_batch_stream, int (*)(void**));
EXPECT_TYPE(dg_last_batch_flags, int (*)(uint32_t*));
EXPECT_TYPE(dg_fallback_count, int (*)(uint64_t*));
EXPECT_TYPE(dg_group_counts, int (*)(uint64_t*));
EXPECT_TYPE(dg_isolation_counts, int (*)(uint64_t*));
EXPECT_TYPE(dg_set_group_size, int (*)(uint32_t));
EXPECT_TYPE(dg_recover_dev, int (*)(const uint8_t*, uint32_t, uint32_t, size_t, const uint8_t*, size_t, uint32_t,
                                    const uint8_t*, uint8_t*, uint8_t*, uint8_t*, uint64_t));
EXPECT_TYPE(dg_verify_partials_dev, int (*)(const uint8_t*, uint32_t, size_t, const uint8_t*, size_t, uint32_t,
                                            const uint8_t*, uint8_t*, uint64_t));
EXPECT_TYPE(dg_recover_verified_dev, int (*)(uint32_t, uint32_t, size_t, uint32_t, const uint8_t*, const uint8_t*,
                                             uint8_t*, uint8_t*, uint8_t*));
EXPECT_TYPE(dg_wait_all, int (*)(void));
EXPECT_TYPE(dg_set_timing, int (*)(int));
EXPECT_TYPE(dg_last_timings, int (*)(const char**, double*, int*, int));

static int fails = 0;
static void expect(const char* what, int got, int want) {
  if (got != want) {
    printf("FAIL %s: %d (want %d)\n", what, got, want);
    ++fails;
  }
}

int main() {
  uint8_t pk[48] = {0xc0}, msg[32] = {0}, sig[96] = {0xc0}, part[98] = {0, 1, 0xc0}, st[4], out[256];
  uint64_t pr[1] = {0}, rr[1] = {1}, u64 = 0;
  uint32_t off[2] = {0, 32}, idx[1] = {0}, flags[2];
  uint16_t ix[1] = {0};
  size_t len = 0;
  const char* names[4];
  double us[4];
  int launches[4];
  // no device in this container: dg_init fails, every compute entry point refuses
  expect("dg_init", dg_init(0) == 0 ? 0 : DG_E_NODEV, DG_E_NODEV);
  expect("dg_device_ready", dg_device_ready(), 0);
  expect("dg_hash_to_g2", dg_hash_to_g2(1, msg, 32, msg, 8, out), DG_E_NODEV);
  expect("dg_sign", dg_sign(1, msg, ix, msg, 32, out), DG_E_NODEV);
  expect("dg_verify", dg_verify(pk, 1, msg, 32, sig, st, 1), DG_E_NODEV);
  expect("dg_verify_beacons", dg_verify_beacons(pk, 1, pr, rr, msg, off, sig, st, 1), DG_E_NODEV);
  expect("dg_check_links", dg_check_links(0, msg, 32, 1, pr, rr, msg, off, sig, st), DG_E_NODEV);
  expect("dg_beacon_messages", dg_beacon_messages(1, pr, rr, msg, off, out), DG_E_NODEV);
  expect("dg_randomness", dg_randomness(1, sig, out), DG_E_NODEV);
  expect("dg_pubpoly_eval", dg_pubpoly_eval(pk, 1, 1, idx, out), DG_E_NODEV);
  expect("dg_verify_partials", dg_verify_partials(pk, 1, 1, msg, 32, 1, part, st, 1), DG_E_NODEV);
  expect("dg_recover", dg_recover(pk, 1, 1, 1, msg, 32, 1, part, out, st, st + 1, 1), DG_E_NODEV);
  expect("dg_recover_dev", dg_recover_dev(pk, 1, 1, 1, msg, 32, 1, part, out, st, st + 1, 1), DG_E_NODEV);
  expect("dg_recover_verified", dg_recover_verified(1, 1, 1, 1, part, st, out, st, st + 1), DG_E_NODEV);
  expect("dg_verify_partials_dev", dg_verify_partials_dev(pk, 1, 1, msg, 32, 1, part, st, 1), DG_E_NODEV);
  expect("dg_recover_verified_dev", dg_recover_verified_dev(1, 1, 1, 1, part, st, out, st, st + 1), DG_E_NODEV);
  expect("dg_verify_beacons_dev", dg_verify_beacons_dev(pk, 1, pr, rr, msg, off, sig, st, 1, nullptr), DG_E_NODEV);
  expect("dg_verify_beacons_dev_async",
         dg_verify_beacons_dev_async(pk, 1, pr, rr, msg, off, sig, st, 1, nullptr, nullptr), DG_E_NODEV);
  void* stream_out = nullptr;
  expect("dg_last_batch_stream", dg_last_batch_stream(&stream_out), DG_E_NODEV);
  expect("dg_last_batch_flags", dg_last_batch_flags(flags), DG_E_NODEV);
  expect("dg_fallback_count", dg_fallback_count(&u64), DG_E_NODEV);
  uint64_t u64x4[4];
  expect("dg_group_counts", dg_group_counts(u64x4), DG_E_NODEV);
  expect("dg_isolation_counts", dg_isolation_counts(u64x4), DG_E_NODEV);
  expect("dg_wait_all", dg_wait_all(), DG_E_NODEV);
  // host-only state works without a device
  int plan_sets = 0, plan_shared = 0;
  expect("dg_queue_plan", dg_queue_plan(4, &plan_sets, &plan_shared), 0);
  expect("dg_queue_plan sets", plan_sets, 8);
  expect("dg_set_timing", dg_set_timing(0), 0);
  expect("dg_last_timings", dg_last_timings(names, us, launches, 4), 0);
  expect("dg_get_hash_dst", dg_get_hash_dst(out, sizeof out, &len), 0);
  expect("default DST", (int)len == 43 && memcmp(out, "BLS_SIG_BLS12381G2_XMD:SHA-256_SSWU_RO_NUL_", 43) == 0, 1);
  expect("dg_set_hash_dst", dg_set_hash_dst((const uint8_t*)"ABC", 3), 0);
  expect("dg_get_hash_dst", dg_get_hash_dst(out, sizeof out, &len), 0);
  expect("switched DST", (int)len == 3 && memcmp(out, "ABC", 3) == 0, 1);
  expect("dst too long", dg_set_hash_dst(out, 256), DG_E_ARG);
  expect("dg_set_group_size", dg_set_group_size(1), 0);
  expect("group size 0", dg_set_group_size(0), DG_E_ARG);
  expect("group size 5", dg_set_group_size(5), DG_E_ARG);
  expect("dg_set_group_size 4", dg_set_group_size(4), 0);
  expect("reset DST", dg_set_hash_dst(nullptr, 0), 0);
  expect("error text", dg_last_error() != nullptr, 1);
  dg_shutdown();
  if (fails) printf("abi_caller: %d failures\n", fails); else printf("abi_caller: ok\n");
  return fails ? 1 : 0;
}
