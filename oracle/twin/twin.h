/* C restatement of the BLS12-381 threshold-BLS path -- TEST INFRASTRUCTURE ONLY (the "CPU twin").
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this library.
 * It is the large-size checker, the chain-fixture generator and the CPU baseline ("port" of the
 * kyber algorithm: one full pairing check per item, PubPoly.Eval recomputed per VerifyPartial,
 * Recover re-verifying every share -- SURVEY.md §8(d)).  It never ships in the product path.
 *
 * Representation (deliberately unlike the HIP kernels): 6 x 64-bit Montgomery limbs with
 * unsigned __int128 products, Jacobian points, textbook tower.  Semantics follow
 * oracle/pyref/tbls.py; status codes match include/drand_gpu.h.
 */
#ifndef DRAND_TWIN_H
#define DRAND_TWIN_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

void twin_init(void);

/* A9: RFC 9380 BLS12381G2_XMD:SHA-256_SSWU_RO_ with the given DST -> compressed 96 B. */
void twin_hash_to_g2(const uint8_t* msg, size_t msg_len, const uint8_t* dst, size_t dst_len, uint8_t out96[96]);
/* A7: sigma = compress(x * H(msg)); scalar is 32 B big-endian (reduced mod r). */
void twin_sign(const uint8_t sk32[32], const uint8_t* msg, size_t msg_len, uint8_t out96[96]);
/* A4: status of bls.Verify(pk, msg, sig) (0 ok, 1 bad sig, 2 sig decode, 4 pk decode). */
int twin_verify(const uint8_t pk48[48], const uint8_t* msg, size_t msg_len, const uint8_t sig96[96]);
/* Batch of A4 over n items with a shared key, `threads` POSIX threads (CPU baseline). */
void twin_verify_batch(const uint8_t pk48[48], size_t n, const uint8_t* msgs, size_t msg_len, const uint8_t* sigs96,
                       uint8_t* status, int threads);
/* A1 */
void twin_beacon_message(const uint8_t* prev_sig, size_t prev_sig_len, uint64_t prev_round, uint64_t round,
                         uint8_t out32[32]);
/* Sequential linked chain: sig_r = x * H(Message(sig_{r-1}, r-1, r)), r = first_round.., sig_{first-1} = seed. */
void twin_gen_chain(const uint8_t sk32[32], const uint8_t* seed, size_t seed_len, uint64_t first_round, size_t n,
                    uint8_t* out_sigs96);
/* A12: PubPoly.Eval(i) for t commits (t x 48 B) -> 48 B; returns 0 or 4 (commit decode error). */
int twin_pubpoly_eval(const uint8_t* commits48, uint32_t t, uint32_t index, uint8_t out48[48]);
/* x * g1, compressed (commit generation) */
void twin_g1_mul_gen(const uint8_t sk32[32], uint8_t out48[48]);
/* A5: VerifyPartial status (3 = bad index) */
int twin_verify_partial(const uint8_t* commits48, uint32_t t, const uint8_t* msg, size_t msg_len,
                        const uint8_t* partial, size_t partial_len);
/* A6: Recover; returns round status (0 ok, 5 not enough). share_status[k] as VerifyPartial, 255 = not examined. */
int twin_recover(const uint8_t* commits48, uint32_t t, uint32_t n, const uint8_t* msg, size_t msg_len,
                 const uint8_t* partials98, uint32_t k, uint8_t out96[96], uint8_t* share_status);
/* Batch Recover over `rounds` rounds of k partials each (CPU baseline), `threads` threads. */
void twin_recover_batch(const uint8_t* commits48, uint32_t t, uint32_t n, size_t rounds, const uint8_t* msgs32,
                        const uint8_t* partials98, uint32_t k, uint8_t* out96, uint8_t* round_status,
                        uint8_t* share_status, int threads);
/* Full pairing e(P, Q) cubed (the twin's final exponentiation computes f^(3(p^12-1)/r)), as 12 Fp2
 * coefficients c[i] (tower slot i = c0.c0,c0.c1,c0.c2,c1.c0,c1.c1,c1.c2), each Fp2 as c0||c1, 48 B BE each. */
int twin_pairing_cubed(const uint8_t g1_48[48], const uint8_t g2_96[96], uint8_t out576[576]);
/* The hash-to-G2 DST used by twin_sign / twin_verify* / twin_recover* (NULL or 0 length: the NUL DST). */
int twin_set_dst(const uint8_t* dst, size_t dst_len);
/* BASELINE configs[0] (C1, beacon/beacon_test.go:41-93) per round: n tbls.Sign partials (share i has index i,
 * shares32 = n x 32 B), Recover over them, VerifyRecovered of the result against commits48[0]; returns the
 * number of rounds that recovered and verified. */
size_t twin_c1_batch(const uint8_t* commits48, uint32_t t, uint32_t n, const uint8_t* shares32, size_t rounds,
                     const uint8_t* msgs32, uint8_t* out96, int threads);
/* instrumented op counter: number of Fp Montgomery multiplications (squarings included) since reset */
void twin_opcount_reset(void);
uint64_t twin_opcount(void);
void twin_opcount_enable(int on);

#ifdef __cplusplus
}
#endif
#endif
