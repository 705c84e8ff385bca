// Driver of the device arithmetic's host build (hostcheck.cpp) under AddressSanitizer + UBSan: the word-wise
// expand_message_xmd, the hash-to-G2 and decompression phase pipelines, the safegcd inversion and a
// pairing check run once each on deterministic inputs.  Test tool only (tests/test_abi.py).
#include <stdint.h>
#include <stdio.h>
#include <string.h>

extern "C" {
int hc_h2f_xmd32_check(const uint8_t* msg32, const uint8_t* dst, uint32_t dl);
int hc_h2c_phases_check(const uint8_t* msg, uint32_t len, const uint8_t* dst, uint32_t dl);
int hc_dec_phases_check(const uint8_t* in96, int subgroup);
void hc_hash_to_g2(const uint8_t* msg, uint32_t n, const uint8_t* dst, uint32_t dl, uint8_t* out96);
void hc_fp_inv(const uint8_t* a48, uint8_t* out_sg48, uint8_t* out_fermat48);
int hc_g2_roundtrip(const uint8_t* in96, uint8_t* out96);
}

int main() {
  static const uint8_t dst[] = "BLS_SIG_BLS12381G2_XMD:SHA-256_SSWU_RO_NUL_";
  int fails = 0;
  uint8_t msg[32], h[96], back[96], a[48], inv1[48], inv2[48];
  for (int j = 0; j < 4; ++j) {
    for (int k = 0; k < 32; ++k) msg[k] = (uint8_t)(17 * j + 31 * k + 5);
    fails += hc_h2f_xmd32_check(msg, dst, 43) != 1;
    fails += hc_h2c_phases_check(msg, 32, dst, 43) != 1;
    hc_hash_to_g2(msg, 32, dst, 43, h);
    fails += hc_dec_phases_check(h, 1) != 1;
    fails += hc_g2_roundtrip(h, back) != 1 || memcmp(h, back, 96) != 0;
    h[50] ^= 1;
    fails += hc_dec_phases_check(h, 0) != 1;
  }
  fails += hc_h2c_phases_check(msg, 7, dst, 43) != 1;
  for (int k = 0; k < 48; ++k) a[k] = (uint8_t)(k * 7 + 1);
  a[0] = 0x11;
  hc_fp_inv(a, inv1, inv2);
  fails += memcmp(inv1, inv2, 48) != 0;
  if (fails) printf("hostcheck_san: %d failures\n", fails); else printf("hostcheck_san: ok\n");
  return fails ? 1 : 0;
}
