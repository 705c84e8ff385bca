"""Generate the committed golden fixtures under tests/golden/ (run once, here; outputs are data).

Everything is computed by the pure-Python oracle (oracle/pyref) and cross-checked against the C twin
(oracle/twin); the two must agree bit-for-bit or generation aborts.  Sources of pinning:
  * kat.json                 -- RFC 9380 expand_message_xmd / hash_to_curve(G2) vectors, an eth2 BLS
                                sign vector, generator encodings, beacon.Message of the 200409 genesis seed
  * reference_g1_keys.json   -- G1 keys held by the reference: deploy/200409/group.toml,
                                demo/docker/data/group.toml and demo/docker/data/*.public (read as text)
  * chain_t3n5.json          -- BASELINE config C1 group (n=5, t=3): 64 linked rounds, partials, Recover
  * adversarial_t3n5.json    -- corrupted partials of every mode with statuses and Recover results
  * g2_decode_edges.json     -- encodings kyber must reject / accept
  * hash_to_g2_nul.json      -- H(m) with drand's DST for 16 messages
Usage: python tests/golden/make_golden.py [--reference /root/reference]
"""
import glob
import hashlib
import json
import os
import re
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from oracle import twin  # noqa: E402
from oracle.pyref import bls12381 as B  # noqa: E402
from oracle.pyref import tbls as T  # noqa: E402
from tools import synthetic as S  # noqa: E402

QUUX_G2 = b"QUUX-V01-CS02-with-BLS12381G2_XMD:SHA-256_SSWU_RO_"
QUUX_XMD = b"QUUX-V01-CS02-with-expander-SHA256-128"
POP = b"BLS_SIG_BLS12381G2_XMD:SHA-256_SSWU_RO_POP_"


def h(b):
    return bytes(b).hex()


def dump(name, obj):
    with open(os.path.join(HERE, name), "w") as f:
        json.dump(obj, f, indent=1, sort_keys=True)
    print("wrote", name)


def kat():
    out = {}
    out["expand_message_xmd"] = [
        {"dst": QUUX_XMD.decode(), "msg": "", "len": 32,
         "expected": "68a985b87eb6b46952128911f2a4412bbc302a9d759667f87f7a21d803f07235"},
        {"dst": QUUX_XMD.decode(), "msg": "abc", "len": 32,
         "expected": "d8ccab23b5985ccea865c6c97b6e5b8350e794e603b4b97902f53a8a0d605615"},
    ]
    for v in out["expand_message_xmd"]:
        assert h(B.expand_message_xmd(v["msg"].encode(), v["dst"].encode(), v["len"])) == v["expected"]
    # RFC 9380 Appendix J.10.1, msg = ""
    px0 = "0141ebfbdca40eb85b87142e130ab689c673cf60f1a3e98d69335266f30d9b8d4ac44c1038e9dcdd5393faf5c41fb78a"
    px1 = "05cb8437535e20ecffaef7752baddf98034139c38452458baeefab379ba13dff5bf5dd71b72418717047f5b0f37da03d"
    py0 = "0503921d7f6a12805e72940b963c0cf3471c7b2a524950ca195d11062ee75ec076daf2d4bc358c4b190c0c98064fdd92"
    py1 = "12424ac32561493f3fe3c260708a12b7c620e7be00099a974e259ddc7d1f6395c3c811cdd19f1e8dbf3e9ecfdcbab8d6"
    pt = B.hash_to_g2(b"", QUUX_G2)
    assert (pt[0].c0, pt[0].c1, pt[1].c0, pt[1].c1) == tuple(int(x, 16) for x in (px0, px1, py0, py1))
    comp = B.g2_compress(pt)
    assert twin.hash_to_g2(b"", QUUX_G2) == comp
    out["hash_to_g2_rfc9380"] = [{"dst": QUUX_G2.decode(), "msg": "", "x0": px0, "x1": px1, "y0": py0, "y1": py1,
                                  "compressed": h(comp)}]
    # eth2 consensus-spec BLS sign vector (POP ciphersuite, same hash-to-curve with another DST)
    sk = 0x263DBD792F5B1BE47ED85F8938C0F29586AF0D3AC7B977F21C278FE1462040E3
    sig = B.g2_compress(B.G2C.mul(B.hash_to_g2(bytes(32), POP), sk))
    exp = ("b6ed936746e01f8ecf281f020953fbf1f01debd5657c4a383940b020b26507f6076334f91e2366c96e9ab279fb5158090352ea1c5b0c"
           "9274504f4f0e7053af24802e51e4568d164fe986834f41e55c8e850ce1f98458c0cfc9ab380b55285a55")
    assert h(sig) == exp
    out["bls_sign_pop"] = [{"sk": "%064x" % sk, "msg": "00" * 32, "dst": POP.decode(), "sig": exp}]
    out["generators"] = {"g1": h(B.g1_compress(B.G1_GEN)), "g2": h(B.g2_compress(B.G2_GEN))}
    seed = bytes.fromhex("770f3c2578a95387b358e02aba5d5008a53ce40047a1fa326dde0dfd0b482a8e")
    m = T.beacon_message(seed, 0, 1)
    assert h(m) == "88015e1b4125cae87e498971b60409667dbadf534ed9e6207004f52d0664f996"
    assert twin.beacon_message(seed, 0, 1) == m
    out["beacon_message"] = [{"prev_sig": h(seed), "prev_round": 0, "round": 1, "expected": h(m)}]
    dump("kat.json", out)


def reference_keys(ref):
    keys = []
    files = [os.path.join(ref, "deploy/200409/group.toml"), os.path.join(ref, "demo/docker/data/group.toml")]
    files += sorted(glob.glob(os.path.join(ref, "demo/docker/data/*.public")))
    for fn in files:
        if not os.path.exists(fn):
            continue
        txt = open(fn).read()
        for hx in re.findall(r'"([0-9a-f]{96})"', txt):
            keys.append({"file": os.path.relpath(fn, ref), "key": hx})
    assert keys, "no reference keys found"
    for k in keys:
        b = bytes.fromhex(k["key"])
        pt = B.g1_decompress(b)  # raises on failure
        assert B.g1_compress(pt) == b
    dump("reference_g1_keys.json", {"source": "G1 keys held by the reference (read as text)", "keys": keys})


def group(t, n):
    coeffs = S.poly_coeffs(t)
    commits = [twin.g1_mul_gen(c) for c in coeffs]
    for c, cm in zip(coeffs, commits):
        assert B.g1_compress(B.G1C.mul(B.G1_GEN, c)) == cm
    shares = [(i, S.share_value(coeffs, i)) for i in range(n)]
    return coeffs, commits, shares


def chain_t3n5():
    t, n = 3, 5
    coeffs, commits, shares = group(t, n)
    x = coeffs[0]
    rounds = []
    prev = S.GENESIS_SEED
    for r in range(1, 65):
        msg = T.beacon_message(prev, r - 1, r)
        sig = twin.sign(x, msg)
        if r <= 4:
            assert T.bls_sign(x, msg) == sig
        rounds.append({"round": r, "prev_round": r - 1, "prev_sig": h(prev), "msg": h(msg), "sig": h(sig),
                       "randomness": h(T.randomness(sig))})
        prev = sig
    # partial signatures and Recover for the first 6 rounds
    partial_rounds = []
    for rd in rounds[:6]:
        msg = bytes.fromhex(rd["msg"])
        parts = [int(i).to_bytes(2, "big") + twin.sign(v, msg) for i, v in shares]
        assert T.tbls_sign(shares[0], msg) == parts[0]
        sig, rs, ss = twin.recover(commits, msg, parts, t, n)
        assert rs == 0 and sig.hex() == rd["sig"]
        partial_rounds.append({"round": rd["round"], "partials": [h(p) for p in parts]})
    # python oracle verifies a sample
    pk = B.g1_decompress(commits[0])
    assert T.bls_verify_status(pk, bytes.fromhex(rounds[0]["msg"]), bytes.fromhex(rounds[0]["sig"])) == 0
    assert T.verify_partial_status(commits, bytes.fromhex(rounds[0]["msg"]),
                                   bytes.fromhex(partial_rounds[0]["partials"][2])) == 0
    dump("chain_t3n5.json", {"t": t, "n": n, "commits": [h(c) for c in commits], "pk": h(commits[0]),
                             "genesis_seed": h(S.GENESIS_SEED), "rounds": rounds, "partial_rounds": partial_rounds,
                             "coeffs": ["%064x" % c for c in coeffs]})
    return coeffs, commits, shares, rounds


def corrupt(mode, part, msg, shares, other_msg, rnd):
    idx = int.from_bytes(part[:2], "big")
    if mode == "wrong_scalar":
        return part[:2] + twin.sign((shares[idx][1] + 1) % B.R, msg)
    if mode == "other_round":
        return part[:2] + twin.sign(shares[idx][1], other_msg)
    if mode == "index_rewritten":
        return ((idx + 1) % len(shares)).to_bytes(2, "big") + part[2:]
    if mode == "random_bytes":
        return part[:2] + hashlib.sha256(b"rnd%d" % rnd).digest() * 3
    if mode == "bitflip_x":
        b = bytearray(part)
        b[2 + 40] ^= 0x04
        return bytes(b)
    if mode == "infinity":
        return part[:2] + bytes([0xC0]) + bytes(95)
    raise ValueError(mode)


MODES = ["wrong_scalar", "other_round", "index_rewritten", "random_bytes", "bitflip_x", "infinity"]


def adversarial(coeffs, commits, shares, rounds):
    t, n = 3, 5
    cases = []
    for k, rd in enumerate(rounds[6:12]):
        msg = bytes.fromhex(rd["msg"])
        other = bytes.fromhex(rounds[0]["msg"])
        parts = [int(i).to_bytes(2, "big") + twin.sign(v, msg) for i, v in shares]
        mode = MODES[k % len(MODES)]
        bad = list(parts)
        bad[0] = corrupt(mode, parts[0], msg, shares, other, rd["round"])
        bad[3] = corrupt(MODES[(k + 1) % len(MODES)], parts[3], msg, shares, other, rd["round"] + 100)
        st = [twin.verify_partial(commits, msg, p) for p in bad]
        # python oracle cross-check of the corrupted ones
        for j in (0, 3):
            assert T.verify_partial_status(commits, msg, bad[j]) == st[j], (mode, j)
        sig, rs, ss = twin.recover(commits, msg, bad, t, n)
        psig, prs, pss = T.recover(commits, msg, bad, t, n, statuses=st)
        assert (sig, rs, ss) == (psig, prs, pss)
        cases.append({"round": rd["round"], "msg": rd["msg"], "modes": [mode, MODES[(k + 1) % len(MODES)]],
                      "partials": [h(p) for p in bad], "verify_status": st, "recover_status": rs,
                      "recover_sig": h(sig) if sig else None, "share_status": ss})
    # not enough: 3 of 5 corrupted
    rd = rounds[12]
    msg = bytes.fromhex(rd["msg"])
    parts = [int(i).to_bytes(2, "big") + twin.sign(v, msg) for i, v in shares]
    bad = [corrupt("wrong_scalar", parts[j], msg, shares, msg, 0) if j < 3 else parts[j] for j in range(5)]
    st = [twin.verify_partial(commits, msg, p) for p in bad]
    sig, rs, ss = twin.recover(commits, msg, bad, t, n)
    assert rs == T.ST_NOT_ENOUGH
    cases.append({"round": rd["round"], "msg": rd["msg"], "modes": ["wrong_scalar x3"], "partials": [h(p) for p in bad],
                  "verify_status": st, "recover_status": rs, "recover_sig": None, "share_status": ss})
    # duplicates collapse: [p0, p0, p1, p2] with t=3 -> 3 collected, 2 distinct -> error
    dup = [parts[3], parts[3], parts[4], parts[0]]
    sig, rs, ss = twin.recover(commits, msg, dup, t, n)
    dst = [twin.verify_partial(commits, msg, p) for p in dup]
    psig, prs, pss = T.recover(commits, msg, dup, t, n, statuses=dst)
    assert rs == prs == T.ST_NOT_ENOUGH
    cases.append({"round": rd["round"], "msg": rd["msg"], "modes": ["duplicate"], "partials": [h(p) for p in dup],
                  "verify_status": dst, "recover_status": rs, "recover_sig": None, "share_status": ss})
    # out-of-order valid partials recover the same signature
    order = [parts[4], parts[2], parts[3]]
    sig, rs, ss = twin.recover(commits, msg, order, t, n)
    assert rs == 0 and sig.hex() == rd["sig"]
    cases.append({"round": rd["round"], "msg": rd["msg"], "modes": ["reordered"], "partials": [h(p) for p in order],
                  "verify_status": [0, 0, 0], "recover_status": 0, "recover_sig": h(sig), "share_status": ss})
    dump("adversarial_t3n5.json", {"t": t, "n": n, "commits": [h(c) for c in commits], "cases": cases})


def g2_edges():
    sig = bytes.fromhex(json.load(open(os.path.join(HERE, "chain_t3n5.json")))["rounds"][0]["sig"])
    cases = []

    def add(name, enc, ok):
        st = twin.verify(bytes(48 * [0]) if False else B.g1_compress(B.G1_GEN), b"x" * 32, enc)
        py_ok = True
        try:
            B.g2_decompress(enc)
        except B.DecodeError:
            py_ok = False
        assert py_ok == ok, name
        cases.append({"name": name, "enc": h(enc), "decodes": ok})

    add("valid", sig, True)
    add("infinity", bytes([0xC0]) + bytes(95), True)
    add("infinity_with_sign_bit", bytes([0xE0]) + bytes(95), False)
    add("infinity_nonzero_body", bytes([0xC0]) + bytes(94) + b"\x01", False)
    add("no_compression_flag", bytes([sig[0] & 0x7F]) + sig[1:], False)
    # x.c1 = p (non-canonical)
    pb = bytearray(B.P.to_bytes(48, "big"))
    pb[0] |= 0x80
    add("x_c1_equals_p", bytes(pb) + sig[48:], False)
    add("x_c0_equals_p", sig[:48] + B.P.to_bytes(48, "big"), False)
    # off-curve and off-subgroup: scan x values
    off_curve = off_sub = None
    for k in range(1, 200):
        x = B.Fp2(k, 1)
        y = (x * x * x + B.G2C.b).sqrt()
        enc = bytearray(x.c1.to_bytes(48, "big") + x.c0.to_bytes(48, "big"))
        enc[0] |= 0x80
        if y is None and off_curve is None:
            off_curve = bytes(enc)
        if y is not None and off_sub is None and not B.g2_in_subgroup((x, y)):
            off_sub = bytes(enc)
        if off_curve and off_sub:
            break
    add("off_curve", off_curve, False)
    add("off_subgroup", off_sub, False)
    flipped = bytearray(sig)
    flipped[0] ^= 0x20
    add("sign_flipped_is_negation", bytes(flipped), True)
    dump("g2_decode_edges.json", {"cases": cases})


def h2c_nul():
    out = []
    for i in range(16):
        m = hashlib.sha256(b"h2c-%d" % i).digest()
        c = twin.hash_to_g2(m)
        if i < 4:
            assert B.g2_compress(B.hash_to_g2(m)) == c
        out.append({"msg": h(m), "h": h(c)})
    dump("hash_to_g2_nul.json", {"dst": twin.DST_NUL.decode(), "vectors": out})


def main():
    ref = "/root/reference"
    if "--reference" in sys.argv:
        ref = sys.argv[sys.argv.index("--reference") + 1]
    kat()
    reference_keys(ref)
    coeffs, commits, shares, rounds = chain_t3n5()
    adversarial(coeffs, commits, shares, rounds)
    g2_edges()
    h2c_nul()


if __name__ == "__main__":
    main()
