"""The kernels' device arithmetic compiled for the host (tests/native/hostcheck.cpp, g++): the same
field/curve/hash code that runs on gfx950, checked on CPU against the oracle and the fixtures."""
import ctypes
import os
import random
import subprocess

import pytest

from oracle.pyref import bls12381 as B
from tests.fixtures import hx, load

HERE = os.path.dirname(os.path.abspath(__file__))
NATIVE = os.path.join(HERE, "native")


@pytest.fixture(scope="module")
def hc():
    subprocess.run(["make", "-s", "-C", NATIVE], check=True)
    return ctypes.CDLL(os.path.join(NATIVE, "libhostcheck.so"))


def test_fp_inv_safegcd_matches_fermat_and_python(hc):
    rng = random.Random(7)
    vals = [0, 1, 2, B.P - 1, B.P - 2, (1 << 380) + 12345] + [rng.randrange(B.P) for _ in range(300)]
    for a in vals:
        sg = ctypes.create_string_buffer(48)
        fe = ctypes.create_string_buffer(48)
        hc.hc_fp_inv(a.to_bytes(48, "big"), sg, fe)
        want = pow(a, B.P - 2, B.P)
        assert int.from_bytes(sg.raw, "big") == want, hex(a)
        assert fe.raw == sg.raw


def test_hash_to_g2_host_build_matches_golden(hc):
    v = load("hash_to_g2_nul.json")
    dst = v["dst"].encode()
    for x in v["vectors"][:4]:
        out = ctypes.create_string_buffer(96)
        m = hx(x["msg"])
        hc.hc_hash_to_g2(m, len(m), dst, len(dst), out)
        assert out.raw.hex() == x["h"]


def test_g2_decode_edges_host_build(hc):
    """ZCash decode + the affine psi subgroup check (curve.h g2_in_subgroup_aff) on the committed edge cases."""
    for c in load("g2_decode_edges.json")["cases"]:
        out = ctypes.create_string_buffer(96)
        assert bool(hc.hc_g2_roundtrip(hx(c["enc"]), out)) == c["decodes"], c["name"]


def test_g2_subgroup_check_host_build_matches_pyref(hc):
    """Uncleared hash outputs (on the curve, almost never in G2) and cleared ones (in G2): the device
    decode's subgroup verdict equals the pyref's [r]P == O test."""
    dst = B.DST_G2
    for i in range(6):
        m = b"subgroup %d" % i
        for pt, in_g2 in ((B.hash_to_g2_uncleared(m, dst), None), (B.hash_to_g2(m, dst), True)):
            enc = B.g2_compress(pt)
            want = B.g2_in_subgroup(pt) if in_g2 is None else in_g2
            out = ctypes.create_string_buffer(96)
            got = bool(hc.hc_g2_roundtrip(enc, out))
            assert got == want, (i, want)
            if got:
                assert out.raw == enc


def test_g2_mul_psi_decomposition_host_build(hc):
    """Recover's lambda * S via the base-|z| digits and psi (curve.h g2_mul_u256_psi) equals 255-bit
    double-and-add, on edge and random scalars."""
    z = 0xD201000000010000
    sig = hx(load("chain_t3n5.json")["rounds"][3]["sig"])
    rng = random.Random(11)
    ks = [0, 1, 2, z - 1, z, z + 1, z * z, z ** 3, z ** 3 - 1, B.R - 1, B.R - z] + [rng.randrange(B.R) for _ in range(12)]
    for k in ks:
        k8 = (ctypes.c_uint32 * 8)(*[(k >> (32 * w)) & 0xFFFFFFFF for w in range(8)])
        assert hc.hc_g2_mul_psi_check(sig, k8) == 1, hex(k)
        assert hc.hc_g2_mul_sac_check(sig, k8) == 1, hex(k)  # the sign-aligned column form
        assert hc.hc_g2_mul_lds_check(sig, k8) == 1, hex(k)  # the LDS-accumulator form of uniform waves


def test_g2_mul_sac_digit_edges_host_build(hc):
    """The sign-aligned column recoding (curve.h g2_mul_u256_psi_sac) at digit edges: even and odd d0,
    zero digits, digits z - 1 (the longest carry chains of the recoding), single high bits."""
    z = 0xD201000000010000
    sig = hx(load("chain_t3n5.json")["rounds"][5]["sig"])
    edge = [0, 1, 2, 3, z - 1, z - 2, 1 << 63, (1 << 63) + 1, 0x5555555555555555, 0xAAAAAAAAAAAAAAAA % z]
    rng = random.Random(12)
    cases = [(a, b, c, d) for a in edge[:6] for b, c, d in ((0, 0, 0), (z - 1, z - 1, z - 1), (1, 0, 1))]
    cases += [tuple(rng.choice(edge) for _ in range(4)) for _ in range(24)]
    for d in cases:
        k = d[0] + d[1] * z + d[2] * z * z + d[3] * z ** 3
        if k >= B.R:
            continue
        k8 = (ctypes.c_uint32 * 8)(*[(k >> (32 * w)) & 0xFFFFFFFF for w in range(8)])
        assert hc.hc_g2_mul_sac_check(sig, k8) == 1, [hex(x) for x in d]


def test_msm4_sac_host_build(hc):
    """The four-point sign-aligned column combination of the group tests (curve.h jac_msm4_sac) in G1 and G2
    equals per-point double-and-add: odd / even / zero / all-ones digits, repeated points (P_0 = P_1) and
    identities."""
    rounds = load("chain_t3n5.json")["rounds"]
    keys = [hx(k) for k in load("groups.json")["t3"]]
    sigs = [hx(rounds[i]["sig"]) for i in range(4)]
    rng = random.Random(13)
    M = (1 << 64) - 1
    digs = [(1, 1, 1, 1), (0, 0, 0, 0), (2, 0, 0, 0), (M, M, M, M), (M - 1, 1, M, 0), (1 << 63, 3, 5, 7)]
    digs += [tuple(rng.getrandbits(64) for _ in range(4)) for _ in range(10)]
    for n, d in enumerate(digs):
        for mask, ss, kk in ((0, sigs, keys[:3] + keys[:1]), (0b0110, sigs, keys[:3] + keys[:1]),
                             (0, [sigs[0], sigs[0]] + sigs[2:], [keys[0], keys[0]] + keys[1:3]), (0b0001, sigs, keys[:3] + keys[:1])):
            dd = (ctypes.c_uint64 * 4)(*d)
            assert hc.hc_msm4_check(b"".join(ss), b"".join(kk), dd, mask) == 1, (n, mask, [hex(x) for x in d])


def test_wordwise_xmd_matches_bytewise(hc):
    """hash_to_field_xmd32 (k_h2c_uncleared's word-wise expand_message_xmd for 32-byte messages) gives the
    byte-wise RFC 9380 path's field elements, for DST lengths across every SHA-256 block boundary."""
    import hashlib

    for dl in (0, 1, 19, 20, 43, 83, 84, 147, 148, 200, 211, 212, 255):
        dst = bytes((7 * k + dl) % 256 for k in range(dl)) if dl != 43 else b"BLS_SIG_BLS12381G2_XMD:SHA-256_SSWU_RO_NUL_"
        for j in range(3):
            msg = hashlib.sha256(b"xmd/%d/%d" % (dl, j)).digest()
            assert hc.hc_h2f_xmd32_check(msg, dst, dl) == 1, (dl, j)


def test_h2c_phases_match_fused(hc):
    """The phase pipeline of hash-to-G2 (drand_amd/csrc/phases.h: p1, exponentiation, p2, exponentiation,
    p3, then the addition of the two maps) lands on the fused hash_to_g2_uncleared's point, for 32-byte
    messages (word-wise expansion) and other lengths (byte-wise)."""
    import hashlib

    dst = b"BLS_SIG_BLS12381G2_XMD:SHA-256_SSWU_RO_NUL_"
    for j in range(40):
        msg = hashlib.sha256(b"ph/%d" % j).digest()
        assert hc.hc_h2c_phases_check(msg, 32, dst, len(dst)) == 1, j
    for ln in (0, 1, 55, 100):
        msg = (hashlib.sha256(b"pl/%d" % ln).digest() * 4)[:ln]
        assert hc.hc_h2c_phases_check(msg, ln, dst, len(dst)) == 1, ln


def test_decode_phases_match_g2_decompress(hc):
    """The decompression phases (k_dec_p1..p3) give g2_decompress's status and point on the golden edge
    cases, the torsion fixtures (with and without the subgroup check) and valid / corrupted signatures."""
    import hashlib

    encs = [hx(c["enc"]) for c in load("g2_decode_edges.json")["cases"]]
    encs += [hx(c["sig"]) for c in load("g2_torsion.json")["cases"]]
    ch = load("chain_t3n5.json")
    for r in ch["rounds"][:16]:
        s = bytearray(hx(r["sig"]))
        encs.append(bytes(s))
        s2 = bytearray(s)
        s2[40] ^= 4
        encs.append(bytes(s2))
        s3 = bytearray(s)
        s3[0] ^= 0x20
        encs.append(bytes(s3))
    for j in range(16):
        b = bytearray(hashlib.sha256(b"rnd/%d" % j).digest() * 3)
        b[0] = (b[0] & 0x3f) | 0x80
        encs.append(bytes(b))
    for e in encs:
        for sub in (0, 1):
            assert hc.hc_dec_phases_check(e, sub) == 1, (e.hex(), sub)


def test_pairing_host_build_matches_twin(hc):
    """The kernels' Miller loop and final exponentiation (pairing.h, with the cyclotomic squarings of the hard
    part) give the CPU twin's e(P, Q)^3 on fixture points, and bls.Verify's verdicts on the golden chain."""
    from oracle import twin

    ch = load("chain_t3n5.json")
    pk = hx(ch["pk"])
    for r in ch["rounds"][:3]:
        sig = hx(r["sig"])
        out = ctypes.create_string_buffer(576)
        assert hc.hc_pairing_cubed(pk, sig, out, 0) == 0
        st, want = twin.pairing_cubed(pk, sig)
        assert st == 0 and out.raw == want
    for i, r in enumerate(ch["rounds"][:4]):
        msg, sig = hx(r["msg"]), hx(ch["rounds"][(i + (i % 2)) % 64]["sig"])
        assert hc.hc_verify(pk, msg, len(msg), sig) == (0 if i % 2 == 0 else 1)


def test_affine_pair_addition_matches_jacobian(hc):
    """The MSM's affine levels (msm.h k_msm_aff_*): chord, tangent, P + (-P) and identity operands through
    curve.h g2_aff_sum with the inverse supplied as the batch inversion would, against the Jacobian addition."""
    c = load("chain_t3n5.json")
    sigs = [hx(r["sig"]) for r in c["rounds"][:6]]
    for i in range(len(sigs) - 1):
        for mode in range(6):
            assert hc.hc_aff_add_check(sigs[i], sigs[i + 1], mode) == 1, (i, mode)


def test_lds_addition_exceptional_cases(hc):
    """curve.h g2_madd_lds / g2_add_lds (Recover's MSM lanes, the keyed chunk sums): a chord, a + a (the tangent) and
    a + (-a) (the identity), the accumulator with Z != 1, against the Jacobian addition."""
    c = load("chain_t3n5.json")
    sigs = [hx(r["sig"]) for r in c["rounds"][:4]]
    for i in range(len(sigs) - 1):
        for mode in range(3):
            for full in (0, 1):
                assert hc.hc_lds_add_check(sigs[i], sigs[i + 1], mode, full) == 1, (i, mode, full)


def test_ck_subgroup_matches_curve_check(hc):
    """checks.h ck_in_subgroup (Recover's k_ck_sub, accumulator in LDS) decides G2 membership as curve.h
    g2_in_subgroup_aff: chain signatures (in G2) and points of E'(Fp2) outside G2 (one bit of x flipped, the
    corrupt.py bitflip_x mode, where the flipped x is still on the curve)."""
    c = load("chain_t3n5.json")
    sigs = [hx(r["sig"]) for r in c["rounds"][:8]]
    seen = {0: 0, 1: 0}
    for sig in sigs:
        assert hc.hc_ck_subgroup_check(sig) == 1
        seen[1] += 1
        for bit in range(8, 40):
            b = bytearray(sig)
            b[95 - bit // 8] ^= 1 << (bit % 8)
            v = hc.hc_ck_subgroup_check(bytes(b))
            assert v in (-1, 0), v
            if v == 0:
                seen[0] += 1
    assert seen[0] >= 20, seen


def test_ck_split_g2_sum_matches_group_combine(hc):
    """checks.h's G2 group sum off the stack (affine 8-entry table in three batched levels, column loop with an LDS-style
    accumulator, batched affine form) equals group_combine's jac_msm4_sac: distinct members, a repeated member (the
    index_rewritten corruption), a member and its negation, the identity, 1..4 live members, edge coefficients."""
    c = load("chain_t3n5.json")
    sigs = [hx(r["sig"]) for r in c["rounds"][:8]]
    neg = lambda s: bytes([s[0] ^ 0x20]) + s[1:]
    ident = bytes([0xc0]) + bytes(95)
    rng = random.Random(5)
    groups = [sigs[0:4], sigs[4:8], [sigs[0], sigs[0], sigs[1], sigs[2]], [sigs[0], neg(sigs[0]), sigs[3], sigs[3]],
              [ident, sigs[1], sigs[2], sigs[3]], [sigs[5], ident, ident, neg(sigs[5])]]
    rhos = [[rng.getrandbits(64) | 1 for _ in range(4)] for _ in range(3)]
    rhos += [[1, 1, 1, 1], [(1 << 64) - 1, 1 << 63, 3, (1 << 64) - 1], [2, 4, 6, 8]]
    for g in groups:
        buf = b"".join(g)
        for rho in rhos:
            arr = (ctypes.c_uint64 * 4)(*rho)
            for nl in (1, 2, 3, 4):
                assert hc.hc_ck_g2_split_check(buf, arr, nl) == 1, (g.index if False else groups.index(g), rho, nl)


def test_fp2_mul_digit_form_matches(hc):
    """field.h fp2_mul_dig (the pipeline's Fp2 product with each operand unpacked once and the Karatsuba sums made
    digit-wise, DG_FP2_DIG) equals fp2_mul on random operands below p and on 0, 1, p - 1."""
    assert hc.hc_fp2_mul_dig_check(ctypes.c_uint64(12345), 3000) == 1


def test_wnaf_digits_host_build(hc):
    """recover.h rc_wnaf: width-5 signed digits (odd, |d| <= 15, >= 5 apart) that evaluate back to the scalar,
    including the 65th position a carry can reach."""
    rng = random.Random(11)
    vals = [0, 1, 15, 16, 17, 31, (1 << 63) - 1, 1 << 63, 0xd201000000010000 - 1, (1 << 64) - 1]
    vals += [rng.getrandbits(64) for _ in range(500)]
    for d in vals:
        assert hc.hc_wnaf_check(ctypes.c_uint64(d)) == 1, hex(d)


def test_lagrange_chunked_products(hc):
    """fr.h lagrange_at_zero (the factors x_m and |x_m - x_j| multiplied in plain 64-bit chunks, one quarter
    Montgomery product per chunk pair, den's sign by parity) equals rc_lambdas' one-product-per-factor form: small
    and consecutive indices (many factors per chunk), indices near 2^32 (one factor per chunk, the chunk boundary
    at every step) and mixtures of both, unsorted."""
    rng = random.Random(29)
    top = (1 << 32) - 2
    sets = [[0], [5], list(range(129)), sorted(rng.sample(range(256), 129)), [top - i for i in range(40)],
            rng.sample(range(top), 64), [0, top, 1, top - 1, 7, 1 << 31, (1 << 31) + 1, 65535, 65536],
            rng.sample(list(range(200)) + [top - i * 977 for i in range(100)], 150)]
    for idx in sets:
        t = len(idx)
        assert hc.hc_lagrange_check((ctypes.c_uint32 * t)(*idx), t) == 1, idx[:8]


@pytest.mark.parametrize("t,seed", [(1, 0), (3, 1), (33, 2), (33, 3), (12, 4), (33, -1), (70, -1)])
def test_recover_msm_host_build(hc, t, seed):
    """recover.h on the host: one Straus MSM per round over the t selected shares (lambdas with one Fr inversion,
    affine odd-multiple tables, four psi-component wNAF schedules, psi combination) equals the sum of the
    per-share products lambda_j S_j (g2_mul_u256_psi), and the lambdas equal lagrange_at_zero's; shares are
    signatures of the committed chain, one of them the identity when t > 3."""
    rounds = load("chain_t3n5.json")["rounds"]
    rng = random.Random(seed + 100)
    sigs = [hx(rounds[rng.randrange(len(rounds))]["sig"]) for _ in range(t)]
    if t > 3:
        sigs[2] = bytes([0xc0]) + bytes(95)  # the identity (a share whose key is the identity)
    # seed -1: the indices 0..t-1 (lambda = +-binomials: the signed digits of the negative ones are small)
    idx = list(range(t)) if seed < 0 else sorted(rng.sample(range(300), t))
    arr = (ctypes.c_uint32 * t)(*idx)
    assert hc.hc_recover_msm_check(b"".join(sigs), arr, t) == 1


@pytest.mark.parametrize("t,seed", [(1, 0), (3, 1), (9, 2), (17, 3), (33, -1)])
def test_recover_sac_host_build(hc, t, seed):
    """recover.h's divergent-round form on the host (sign-aligned tables in three affine levels, one doubling per
    column shared by groups of 8 shares, even-digit corrections, group sums) equals sum_j lambda_j S_j; one share
    is the identity when t > 3."""
    rounds = load("chain_t3n5.json")["rounds"]
    rng = random.Random(seed + 200)
    sigs = [hx(rounds[rng.randrange(len(rounds))]["sig"]) for _ in range(t)]
    if t > 3:
        sigs[1] = bytes([0xc0]) + bytes(95)
    idx = list(range(t)) if seed < 0 else sorted(rng.sample(range(256), t))
    assert hc.hc_recover_sac_check(b"".join(sigs), (ctypes.c_uint32 * t)(*idx), t) == 1



def test_karabina_exponentiation_matches_granger_scott(hc):
    """pairing.h cyc_exp_z (compressed squarings, one batched Fp2 inversion for the six decompressions) equals the
    Granger-Scott square-and-multiply chain on cyclotomic elements, and the all-zero-denominator fallback (a = 1)
    returns 1."""
    hc.hc_cyc_exp_check.restype = ctypes.c_int
    hc.hc_cyc_exp_check.argtypes = [ctypes.c_uint64, ctypes.c_uint32]
    assert hc.hc_cyc_exp_check(0xD1CE5EED, 24) == 0


def test_check_pipeline_matches_pair_check(hc):
    """Recover's pairing-check pipeline (checks.h: per-round lines without the G1 point, the Miller value from two
    line tables -- also as two single-pair values multiplied, with the lines from the tables and computed in the lane
    (ck_miller1_fly, the isolation's k_xg_miller) -- the final exponentiation with in-lane
    inversions, the compressed chains and the fused next factors) equals
    final_exp_cubed(miller_loop<2>) on the host: valid and invalid (key, H, sigma) triples of the golden chain, each
    pair dropped alone (np = 1, 2) and both.  k_ck_miller's digit-form loop (fpd.h, checks.h ck_miller_col) must give the same
    Miller value with every digit-form bound holding."""
    from tests.fixtures import chain, chain_arrays

    c = chain()
    _, _, _, sigs, msgs = chain_arrays(c)
    pk = hx(c["pk"])
    dst = b"BLS_SIG_BLS12381G2_XMD:SHA-256_SSWU_RO_NUL_"
    hc.hc_ck_pipeline_check.restype = ctypes.c_int
    for i in range(6):
        out = ctypes.create_string_buffer(96)
        hc.hc_hash_to_g2(bytes(msgs[i]), 32, dst, len(dst), out)
        h = out.raw
        for sig, np_ in ((bytes(sigs[i]), 3), (bytes(sigs[i + 1]), 3), (bytes(sigs[i]), 1), (bytes(sigs[i]), 2)):
            assert hc.hc_ck_pipeline_check(pk, h, sig, np_) == 1, (i, np_)


def test_digit_form_fp12_matches_field(hc):
    """fpd.h (the Miller loop's digit form: 14 x 28-bit digits through whole Fp12 operations, fat multiples of p for
    subtractions, one reduction per output) equals field.h's fp12_sqr and fp12_mul_014, alone and chained, on random
    elements and on the extreme one, with the bounds asserted in every product, subtraction and reduction."""
    hc.hc_fd_check.restype = ctypes.c_int
    hc.hc_fd_check.argtypes = [ctypes.c_uint64, ctypes.c_int]
    assert hc.hc_fd_check(0xF0D5EED, 200) == 0


def test_xr_quad_sum_matches_double_and_add(hc):
    """xr.h xq_sum4 -- the cross-round isolation's quad sums sum rho_i P_i (k_xq_sum: the affine 8-entry table built in
    the lane, one Fp inversion per level, the sign-aligned column loop) -- equals double-and-add per point: distinct
    points, a repeated point, a point and its negation, the identity, 1..4 live members, edge coefficients."""
    c = load("chain_t3n5.json")
    sigs = [hx(r["sig"]) for r in c["rounds"][:8]]
    neg = lambda s: bytes([s[0] ^ 0x20]) + s[1:]
    ident = bytes([0xc0]) + bytes(95)
    rng = random.Random(11)
    groups = [sigs[0:4], sigs[4:8], [sigs[0], sigs[0], sigs[1], sigs[2]], [sigs[0], neg(sigs[0]), sigs[3], sigs[3]],
              [ident, sigs[1], sigs[2], sigs[3]], [sigs[5], ident, ident, neg(sigs[5])], [sigs[6]] * 4]
    rhos = [[rng.getrandbits(64) | 1 for _ in range(4)] for _ in range(3)]
    rhos += [[1, 1, 1, 1], [(1 << 64) - 1, 1 << 63, 3, (1 << 64) - 1], [2, 4, 6, 8], [5, 5, (1 << 64) - 5, 5]]
    hc.hc_xq_sum_check.restype = ctypes.c_int
    for gi, g in enumerate(groups):
        buf = b"".join(g)
        for rho in rhos:
            arr = (ctypes.c_uint64 * 4)(*rho)
            for nl in (1, 2, 3, 4):
                assert hc.hc_xq_sum_check(buf, arr, nl) == 1, (gi, rho, nl)
