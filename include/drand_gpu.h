/* drand_gpu.h -- C-ABI of the MI355X threshold-BLS engine (libdrandgpu.so).
 *
 * The drop-in boundary for drand's signature scheme: drand reaches it through `key.Scheme`
 * (key/curve.go:30, `tbls.NewThresholdSchemeOnG2(Pairing)`, a kyber `sign.ThresholdScheme`), which the
 * beacon is handed via `beacon.Config.Scheme` (beacon/beacon.go:33, set at core/drand.go:335).  A Go
 * `gpu/` package implements that interface with cgo calls into the functions below;
 * points cross the boundary only as bytes (kyber `MarshalBinary`: 48 B G1, 96 B G2, 98 B partials =
 * BE16 index || 96 B G2).
 *
 * Conventions
 *   - Return value: 0 on success, < 0 on a fatal error (see DG_E_*); dg_last_error() has the text.
 *   - Per-item results are written to caller-owned `status` arrays (DG_ST_*).  Error *text* parity
 *     with kyber is not provided; nil / non-nil parity is: status != DG_ST_OK <=> kyber returns an error.
 *   - Buffers are borrowed for the duration of the call only (cgo pointer rules); nothing is retained.
 *   - Thread-safe: calls on one process-wide context are serialised by a mutex (beacon/beacon.go:124
 *     calls the scheme from concurrent gRPC handlers).
 *   - All arithmetic runs in HIP kernels on the selected MI355X (gfx950).  There is no CPU fallback:
 *     without a device every compute entry point returns DG_E_NODEV.
 *   - `msg_len` is the per-item message length (drand: 32 B SHA-256 outputs); all items of one call
 *     share it.  Messages are laid out back to back (n x msg_len bytes).
 *   - Verdicts of the batch paths are exact for every rejected item and probabilistic for accepted ones:
 *     a batch (or a group test: up to 4 shares of one Recover / VerifyPartial round, or 4..16 rounds of a
 *     failed chain batch) that passes its random-linear-combination equation accepts all its members, and a
 *     bad member survives with probability <= 2^-63 (64-bit coefficients bound to the batch contents,
 *     DESIGN.md §4.4).  A failed equation splits its members into smaller group tests and, last, single
 *     pairing checks: every rejection is a single check's.  dg_set_group_size(1) makes the multi-key per-item
 *     pass (Recover, VerifyPartial) use single checks only.
 */
#ifndef DRAND_GPU_H
#define DRAND_GPU_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* per-item status */
#define DG_ST_OK 0
#define DG_ST_BAD_SIG 1      /* pairing check failed                               */
#define DG_ST_SIG_DECODE 2   /* sigma: bad flags / non-canonical / off-curve / off-subgroup */
#define DG_ST_BAD_INDEX 3    /* partial signature too short to carry an index      */
#define DG_ST_PK_DECODE 4    /* public key / commitment does not decode             */
#define DG_ST_NOT_ENOUGH 5   /* Recover: fewer than t distinct valid shares         */
#define DG_ST_NOT_EXAMINED 255 /* Recover: partial after the t-th collected one       */

/* fatal return codes */
#define DG_E_NODEV (-1)
#define DG_E_ARG (-2)
#define DG_E_HIP (-3)
#define DG_E_NOMEM (-4)

/* Select the HIP device this process uses (one process per GPU).  Idempotent for the same device. */
int dg_init(int device);
void dg_shutdown(void);
const char* dg_last_error(void);
/* 1 if the library runs on a gfx950 device after dg_init, else 0 */
int dg_device_ready(void);

/* The hash-to-G2 domain-separation tag of every signing / verifying entry point (dg_sign, dg_verify*,
 * dg_verify_partials, dg_recover).  The suite's hash lives in github.com/drand/bls12-381 v0.2.0 (key/curve.go:4,12),
 * whose DST / draft version no file in the reference pins; it defaults to the RFC 9380
 * "BLS_SIG_BLS12381G2_XMD:SHA-256_SSWU_RO_NUL_" and a maintainer can switch it at run time, without a rebuild.
 * dst_len 0 restores the default; at most 255 bytes.  Process-wide; batches already enqueued keep theirs. */
int dg_set_hash_dst(const uint8_t* dst, size_t dst_len);
/* The current DST: *len = its length, min(cap, len) bytes copied to out (out may be NULL). */
int dg_get_hash_dst(uint8_t* out, size_t cap, size_t* len);

/* A9 -- hash-to-G2 (RFC 9380 XMD:SHA-256_SSWU_RO_ with `dst`), compressed 96 B per message.
 * Replaces kyber's hashablePoint.Hash used inside bls.Sign / bls.Verify [UPSTREAM]. */
int dg_hash_to_g2(size_t n, const uint8_t* msgs, size_t msg_len, const uint8_t* dst, size_t dst_len, uint8_t* out96);

/* A7 -- tbls.Sign (beacon/beacon.go:433): out = BE16(index) || compress(x_i * H(msg)), 98 B each.
 * scalars32: n x 32 B big-endian (reduced mod r).  If `index` is NULL the 96 B bls.Sign output is written. */
int dg_sign(size_t n, const uint8_t* scalars32, const uint16_t* index, const uint8_t* msgs, size_t msg_len,
            uint8_t* out);

/* A3/A4 -- tbls.VerifyRecovered / bls.Verify batch against one key (beacon/beacon.go:494,575,
 * beacon/chain.go:70, core/client_public.go:116).  Random-linear-combination multi-pairing with one
 * shared final exponentiation; on a failed batch the bad items are isolated on the device by group tests
 * across items (groups of 16, then every item of a failed group alone): a rejected item failed its own exact
 * check, an accepted item is valid except with probability <= 2^-63 (see Conventions).  `seed` keys the 64-bit
 * RLC coefficients (0: from the OS). */
int dg_verify(const uint8_t pk48[48], size_t n, const uint8_t* msgs, size_t msg_len, const uint8_t* sigs96,
              uint8_t* status, uint64_t seed);

/* A1 + A3 -- beacon.VerifyBeacon over a batch (beacon/chain.go:65-71): msg = SHA256(BE64(prev_round) ||
 * prev_sig || BE64(round)) computed on the device, then as dg_verify.  prev_sig of item i is
 * prev_sigs[prev_sig_off[i] .. prev_sig_off[i+1]) (96 B, or the 32 B genesis seed for round 1). */
int dg_verify_beacons(const uint8_t pk48[48], size_t n, const uint64_t* prev_round, const uint64_t* round,
                      const uint8_t* prev_sigs, const uint32_t* prev_sig_off, const uint8_t* sigs96,
                      uint8_t* status, uint64_t seed);

/* A13 -- chain-link check of syncFrom (beacon/beacon.go:561-573) for items i = 0..n-1 against the
 * previous item (item 0 against cur_round / cur_sig): 0 = linked, 1 = broken. */
int dg_check_links(uint64_t cur_round, const uint8_t* cur_sig, size_t cur_sig_len, size_t n,
                   const uint64_t* prev_round, const uint64_t* round, const uint8_t* prev_sigs,
                   const uint32_t* prev_sig_off, const uint8_t* sigs96, uint8_t* link_status);

/* A1 -- beacon.Message batch (beacon/chain.go:86-94). */
int dg_beacon_messages(size_t n, const uint64_t* prev_round, const uint64_t* round, const uint8_t* prev_sigs,
                       const uint32_t* prev_sig_off, uint8_t* out32);

/* A2 -- RandomnessFromSignature batch (beacon/chain.go:52-55): SHA-256 of each 96 B signature. */
int dg_randomness(size_t n, const uint8_t* sigs96, uint8_t* out32);

/* A12 -- share.PubPoly.Eval batch: Horner over t G1 commits at x = index + 1, compressed 48 B. */
int dg_pubpoly_eval(const uint8_t* commits48, uint32_t t, size_t n, const uint32_t* index, uint8_t* out48);

/* A5 -- tbls.VerifyPartial batch (beacon/beacon.go:148): `rounds` messages, k partials (98 B) per round,
 * status[r*k + j].  X_i = PubPoly.Eval(i) is computed once per distinct index on the device. */
int dg_verify_partials(const uint8_t* commits48, uint32_t t, size_t rounds, const uint8_t* msgs, size_t msg_len,
                       uint32_t k, const uint8_t* partials98, uint8_t* status, uint64_t seed);

/* A6 -- tbls.Recover batch (beacon/beacon.go:488): per round, the first t partials (input order) that
 * pass VerifyPartial, deduplicated by index, Lagrange-interpolated at 0 on G2.  round_status[r] is
 * DG_ST_OK or DG_ST_NOT_ENOUGH; share_status[r*k + j] is the VerifyPartial status of partials Recover
 * examined and DG_ST_NOT_EXAMINED for the rest.  After a failed batch equation the examined prefix is
 * checked by group tests (see Conventions: an accepted member is valid except with probability <= 2^-63;
 * rejected members and every member of a failed group get their own exact check). */
int dg_recover(const uint8_t* commits48, uint32_t t, uint32_t nshares, size_t rounds, const uint8_t* msgs,
               size_t msg_len, uint32_t k, const uint8_t* partials98, uint8_t* out_sig96, uint8_t* round_status,
               uint8_t* share_status, uint64_t seed);

/* A6 on the live round (beacon/beacon.go:472-494): tbls.Recover for partials whose VerifyPartial verdicts the
 * caller already holds -- ProcessBeacon verified every partial at beacon/beacon.go:148 before the round cache
 * (beacon/round_cache.go:113-119) kept it, and kyber's Recover (:488) verifies each again.  verified_status[r*k + j]
 * is that verdict (DG_ST_OK = valid); a non-OK partial is skipped exactly as Recover skips a failing one.
 * Per round: the first t partials with an OK verdict (input order), deduplicated by index, Lagrange-interpolated
 * at 0 on G2; no pairing is computed.  Outputs as dg_recover.  The caller vouches for the verdicts, and each
 * must have been computed against THIS round's message: ProcessBeacon verifies a packet against the message
 * built from the packet's own PreviousSig (beacon/beacon.go:146-148) while the round cache admits partials
 * by PreviousRound alone (round_cache.go:40-48), so a verdict for another prev-sig is not a verdict for this
 * message -- the Go wrapper (gpu.Scheme.RecoverVerified) re-verifies such partials before calling this. */
int dg_recover_verified(uint32_t t, uint32_t nshares, size_t rounds, uint32_t k, const uint8_t* partials98,
                        const uint8_t* verified_status, uint8_t* out_sig96, uint8_t* round_status,
                        uint8_t* share_status);

/* ---- device-resident variants (bench / multi-GPU path): pointers are device memory on the current
 * device, work is enqueued on `stream` (a hipStream_t; NULL = the library's stream) and completes before
 * return.  Semantics as the host versions. */
int dg_verify_beacons_dev(const uint8_t* pk48_host, size_t n, const uint64_t* d_prev_round, const uint64_t* d_round,
                          const uint8_t* d_prev_sigs, const uint32_t* d_prev_sig_off, const uint8_t* d_sigs96,
                          uint8_t* d_status, uint64_t seed, void* stream);
/* dg_recover with messages, partials and outputs in device memory (commits48 stays a host buffer): the
 * multi-GPU Recover path, whose outputs go straight into the RCCL all-gather.  Completes before return. */
int dg_recover_dev(const uint8_t* commits48, uint32_t t, uint32_t nshares, size_t rounds, const uint8_t* d_msgs,
                   size_t msg_len, uint32_t k, const uint8_t* d_partials98, uint8_t* d_out_sig96,
                   uint8_t* d_round_status, uint8_t* d_share_status, uint64_t seed);

/* dg_verify_partials with messages, partials and statuses in device memory (commits48 stays a host buffer):
 * VerifyPartial of every incoming partial as ProcessBeacon does (beacon/beacon.go:148), HBM-resident.  Completes
 * before return. */
int dg_verify_partials_dev(const uint8_t* commits48, uint32_t t, size_t rounds, const uint8_t* d_msgs, size_t msg_len,
                           uint32_t k, const uint8_t* d_partials98, uint8_t* d_status, uint64_t seed);
/* dg_recover_verified with partials, verdicts and outputs in device memory: the Lagrange half of the live round
 * (beacon/beacon.go:488) after dg_verify_partials_dev.  Completes before return. */
int dg_recover_verified_dev(uint32_t t, uint32_t nshares, size_t rounds, uint32_t k, const uint8_t* d_partials98,
                            const uint8_t* d_verified_status, uint8_t* d_out_sig96, uint8_t* d_round_status,
                            uint8_t* d_share_status);

/* Asynchronous device-resident VerifyBeacon batch (the streaming form of syncFrom's catch-up,
 * beacon/beacon.go:529-607): enqueues the batch on the next of the library's rotating workspace sets and
 * returns without waiting, so consecutive batches overlap (one batch's Miller loops and final
 * exponentiation -- a few workgroups -- run beside the next batch's hashing and decoding).  in_stream
 * (may be NULL): the inputs are ready when this stream reaches the call; done_stream (may be NULL):
 * made to wait for the batch's completion (e.g. before an all-gather of the statuses).  d_status is
 * final after dg_wait_all() or once done_stream passes that point.  The device buffers must stay
 * untouched until then. */
int dg_verify_beacons_dev_async(const uint8_t* pk48_host, size_t n, const uint64_t* d_prev_round,
                                const uint64_t* d_round, const uint8_t* d_prev_sigs, const uint32_t* d_prev_sig_off,
                                const uint8_t* d_sigs96, uint8_t* d_status, uint64_t seed, void* in_stream,
                                void* done_stream);
/* The workspace plan dg_init uses for a hardware queue count (GPU_MAX_HW_QUEUES; HIP's default 4): *sets workspace
 * sets (batches in flight; DG_SETS overrides) and whether the per-item pass runs on each set's own stream (1, at
 * every queue count since the check pipeline replaced the large-scratch per-item kernels).  Host-only, no device
 * needed.  (No reference counterpart.) */
int dg_queue_plan(int hw_queues, int* sets, int* per_item_on_set_streams);
/* The HIP stream (hipStream_t) the most recent dg_verify_beacons_dev_async batch completes on (its high-priority tail
 * stream).  Work the caller enqueues there runs after that batch with no cross-stream wait: with fewer
 * hardware queues than streams (GPU_MAX_HW_QUEUES, HIP's default 4) a wait queued on a shared queue holds every stream
 * behind it, so a short consumer of one batch's statuses (a bitmap pack, an all-gather, a copy) is cheapest on this
 * stream.  The stream is SHARED and HIGH PRIORITY: the library has 4 tail streams and consecutive batches end on
 * different ones, so the batch four batches later ends on the same one, and whatever the caller enqueues there runs
 * at high priority and ahead of that later batch's tail (its Miller loops, final exponentiation and isolation).  Keep it short; for long work record
 * an event here and wait for it on a stream of the caller's.  The stream stays owned by the library (valid until
 * dg_shutdown); DG_E_ARG before the first asynchronous batch.  (No reference counterpart: drand verifies beacons one
 * at a time, beacon/chain.go:65-71.) */
int dg_last_batch_stream(void** out);
/* Diagnostics of the most recent verification batch: out2[0] = 1 if the random-linear-combination
 * batch equation held, out2[1] = 1 if some item was checked on its own (duplicate key cell).  A valid
 * batch must pass on the batch path; the per-item fallback only decides failures. */
int dg_last_batch_flags(uint32_t* out2);
/* Number of batches since dg_init whose batch equation failed or that isolated items, i.e. ran the
 * per-item pass (waits for batches in flight).  A stream of valid batches keeps it at 0. */
int dg_fallback_count(uint64_t* out);
/* Recover's per-item pass since dg_init (waits for batches in flight): out4[m - 1] = checks of m shares of
 * one round at once (m = 1: a share's own bls.Verify; m = 2..4: a random-linear-combination group test). */
int dg_group_counts(uint64_t* out4);
/* The isolation of failed single-key batches (dg_verify, dg_verify_beacons*) since dg_init (waits for batches in
 * flight): out3[0] = group tests of 4..256 rounds (16 by default), out3[1] = 0 (the round-5 quad level, removed),
 * out3[2] = single bls.Verify checks (beacon/chain.go:65-71 decides every round alone; a failed batch equation splits
 * its rounds this way). */
int dg_isolation_counts(uint64_t* out3);
/* Shares per group test in Recover's per-item pass: 1..4 (default 4, or the DG_GROUP environment variable);
 * 1 = every examined share gets its own exact pairing check.  Process-wide. */
int dg_set_group_size(uint32_t m);
/* Wait for every batch enqueued by the asynchronous entry points. */
int dg_wait_all(void);

/* Per-kernel HIP-event timing on the launch stream (off by default); resets the accumulated table. */
int dg_set_timing(int on);

/* kernel timing of the last call on this context: number of entries written (<= cap);
 * names/us are kernel-name pointers (static strings) and average microseconds per launch. */
int dg_last_timings(const char** names, double* us, int* launches, int cap);

#ifdef __cplusplus
}
#endif
#endif
