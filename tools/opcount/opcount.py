"""Per-unit Montgomery multiplication/squaring counts of each verify-path kernel, from the instrumented
host build of the device arithmetic (liboc.so), averaged over the committed 64-round chain fixture.
Writes profiles/opcounts.json, which bench.py reads to convert kernel time into multiply-adds/s.
MACs (the algorithmic unit): one Montgomery multiplication or squaring M = 300 32x32-bit
multiply-adds, 2 * 12^2 + 12 for 12-limb CIOS, a squaring counted as a multiplication.  vmad (the issue
unit): the v_mad_u64_u32 the radix-2^28 kernels of fp28.h execute, 392 per multiplication and 301 per
squaring (14 x 14 column products + 14 x 14 reduction products; the squaring doubles the off-diagonal
terms), counted in the disassembly (profiles/r3_vmad_counts.txt)."""
import ctypes
import hashlib
import json
import os
import random
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
MAC_MUL, MAC_SQR = 300, 300
VMAD_MUL, VMAD_SQR = 392, 301
# one safegcd inversion (field.h fp_inv): 37 batches x 13 limbs x (6 + 4) signed 32x32->64 multiply-adds
MAC_INV = 37 * 13 * 10
DST = b"BLS_SIG_BLS12381G2_XMD:SHA-256_SSWU_RO_NUL_"


def main():
    subprocess.run(["make", "-s", "-C", HERE], check=True)
    L = ctypes.CDLL(os.path.join(HERE, "liboc.so"))
    c = json.load(open(os.path.join(ROOT, "tests", "golden", "chain_t3n5.json")))
    rounds = c["rounds"]
    pk = bytes.fromhex(c["pk"])
    o = (ctypes.c_uint64 * 3)()
    acc = {}

    def add(name, n=1):
        m, s, v = o[0], o[1], o[2]
        a = acc.setdefault(name, [0, 0, 0, 0])
        a[0] += m
        a[1] += s
        a[2] += v
        a[3] += n

    for i, r in enumerate(rounds):
        msg = bytes.fromhex(r["msg"])
        sig = bytes.fromhex(r["sig"])
        alpha = int.from_bytes(hashlib.sha256(b"a%d" % i).digest()[:8], "big") | 1
        L.oc_h2c_uncleared(msg, 32, DST, len(DST), o)
        add("k_h2c_uncleared")
        ph = (ctypes.c_uint64 * 15)()
        L.oc_h2c_phases(msg, DST, len(DST), ph)
        for q, name, n in ((0, "k_h2c_p1a+p1b", 1), (1, "k_exp_pm3d4", 1), (2, "k_h2c_p2", 2), (3, "k_h2c_p3", 2),
                           (4, "k_h2c_p4a+p4b", 1)):
            o[0], o[1], o[2] = ph[3 * q], ph[3 * q + 1], ph[3 * q + 2]
            add(name, n)  # per round (p1, p4), per map item (p2, p3), per exponentiation
        dp = (ctypes.c_uint64 * 12)()
        assert L.oc_dec_phases(sig, dp) == 1
        for q, name in ((0, "k_dec_p1"), (2, "k_dec_p2"), (3, "k_dec_p3")):
            o[0], o[1], o[2] = dp[3 * q], dp[3 * q + 1], dp[3 * q + 2]
            add(name)
        assert L.oc_decode_g2(sig, 0, o) == 1
        add("k_decode_items")  # one key, one item per round: subgroup check batched (msm.h)
        assert L.oc_decode_g2(sig, 1, o) == 1
        add("k_decode_items[+subgroup]")
        L.oc_round_combine(msg, 32, DST, len(DST), sig, ctypes.c_uint64(alpha), o)
        add("k_round_combine (k > 1)")
        L.oc_scale_item(sig, ctypes.c_uint64(alpha), o)
        add("k_kmsm_beta (per key)")
        nxt = bytes.fromhex(rounds[(i + 1) % len(rounds)]["sig"])
        L.oc_g2_add(sig, nxt, o)
        add("k_sum_rows")
        L.oc_g2_add_aff(sig, nxt, o)
        add("k_msm_chunks[mixed add]")
        lam = (ctypes.c_uint32 * 8)(*[int.from_bytes(hashlib.sha256(b"l%d%d" % (i, w)).digest()[:4], "little")
                                      for w in range(7)] + [0x3fffffff])
        L.oc_recover_term(sig, lam, o)
        add("k_recover_terms")
        if i < 8:
            L.oc_verify_item(pk, msg, 32, DST, len(DST), sig, o)
            add("pair_check (one bls.Verify, single lane)")
            nxt4 = b"".join(bytes.fromhex(rounds[(i + q) % len(rounds)]["sig"]) for q in range(4))
            ck = (ctypes.c_uint64 * 24)()
            for m in range(1, 5):
                L.oc_check_pipeline(pk * m, msg, DST, len(DST), nxt4[:96 * m], m, ck)
                for q, kname in ((0, "k_ck_prep[%d]" % m), (1, "k_ck_lines2"), (2, "k_ck_miller"), (3, "k_ck_easy"),
                                 (4, "k_ck_expsq (5 per check)"), (5, "k_ck_expdec (5 per check)"), (6, "k_ck_final"),
                                 (7, "k_ck_round_lines (per round)")):
                    if m > 1 and not kname.startswith("k_ck_prep"):
                        continue  # the same per check whatever m (the Miller loop's G1 point only)
                    o[0], o[1], o[2] = ck[3 * q], ck[3 * q + 1], ck[3 * q + 2]
                    add(kname)
                    if q == 7:
                        add("k_xg_hlines")  # the same work per cross-round check (h_eff and 68 lines)
            xr = (ctypes.c_uint64 * 9)()
            L.oc_xr_units(nxt4, 4, xr)
            for q, kname in ((0, "k_xq_sum (per quad side)"), (1, "k_xg_prep[level 1, 4 quads]"),
                             (2, "k_xg_prep[level 2]")):
                o[0], o[1], o[2] = xr[3 * q], xr[3 * q + 1], xr[3 * q + 2]
                add(kname)
            L.oc_batch_final(pk, sig, nxt, o)
            add("k_pair_miller+k_final_check")
    # Recover's per-round MSM at n = 64, t = 33: the C3 index set (0..32: every share valid, input order) and a
    # random set of 33 of 64 (lambda without structure); per round
    rng = random.Random(5)
    sig33 = b"".join(bytes.fromhex(rounds[q % len(rounds)]["sig"]) for q in range(33))
    for name, idx in (("", list(range(33))), ("[random set]", sorted(rng.sample(range(64), 33)))):
        rc = (ctypes.c_uint64 * 9)()
        L.oc_recover_msm(sig33, (ctypes.c_uint32 * 33)(*idx), 33, rc)
        for q, kname in ((0, "k_rc_tables"), (1, "k_rc_straus"), (2, "k_rc_combine")):
            o[0], o[1], o[2] = rc[3 * q], rc[3 * q + 1], rc[3 * q + 2]
            add(kname + name)
    # the divergent-round form at n = 256, t = 129 (C5: rounds with corrupted shares select scattered index sets)
    sig129 = b"".join(bytes.fromhex(rounds[q % len(rounds)]["sig"]) for q in range(129))
    rs = (ctypes.c_uint64 * 9)()
    L.oc_recover_sac(sig129, (ctypes.c_uint32 * 129)(*sorted(rng.sample(range(256), 129))), 129, rs)
    for q, kname in ((0, "k_rs_tables"), (1, "k_rs_sac"), (2, "k_rs_combine")):
        o[0], o[1], o[2] = rs[3 * q], rs[3 * q + 1], rs[3 * q + 2]
        add(kname)
    out = {"mac_per_mul": MAC_MUL, "mac_per_sqr": MAC_SQR, "mac_per_inv": MAC_INV, "vmad_per_mul": VMAD_MUL,
           "vmad_per_sqr": VMAD_SQR, "basis": "BASELINE.md: 300 multiply-adds per Montgomery product M",
           "sample": "tests/golden/chain_t3n5.json (64 rounds)", "per_unit": {}}
    for k, (m, s, v, n) in acc.items():
        out["per_unit"][k] = {"mul": m / n, "sqr": s / n, "inv": v / n, "M": (m + s) / n,
                              "macs": (m * MAC_MUL + s * MAC_SQR + v * MAC_INV) / n,
                              "vmad": (m * VMAD_MUL + s * VMAD_SQR + v * MAC_INV) / n}
    out["per_unit"]["k_key_accum"] = out["per_unit"]["k_sum_rows"]
    with open(os.path.join(ROOT, "profiles", "opcounts.json"), "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
    for k, v in sorted(out["per_unit"].items()):
        print("%-28s M=%9.1f  MACs=%12.0f" % (k, v["M"], v["macs"]))


if __name__ == "__main__":
    main()
