"""Oracle pinning (CPU): the pure-Python restatement and the C twin against the committed known-answer
vectors (RFC 9380, eth2 BLS, the reference's own G1 keys, beacon.Message of the 200409 genesis seed) and
against each other.  Neither touches the product path; both are the checkers of tests/test_gpu_*.py."""
import hashlib
import os

import pytest

from oracle import twin
from oracle.pyref import bls12381 as B
from oracle.pyref import tbls as T
from tests.fixtures import chain, chain_arrays, hx, load

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_expand_message_xmd_rfc9380():
    for v in load("kat.json")["expand_message_xmd"]:
        assert B.expand_message_xmd(v["msg"].encode(), v["dst"].encode(), v["len"]).hex() == v["expected"]


def test_hash_to_g2_rfc9380_pyref_and_twin():
    for v in load("kat.json")["hash_to_g2_rfc9380"]:
        pt = B.hash_to_g2(v["msg"].encode(), v["dst"].encode())
        assert (pt[0].c0, pt[0].c1, pt[1].c0, pt[1].c1) == tuple(int(v[k], 16) for k in ("x0", "x1", "y0", "y1"))
        assert B.g2_compress(pt).hex() == v["compressed"]
        assert twin.hash_to_g2(v["msg"].encode(), v["dst"].encode()).hex() == v["compressed"]


def test_bls_sign_eth2_vector():
    for v in load("kat.json")["bls_sign_pop"]:
        sk = int(v["sk"], 16)
        msg = hx(v["msg"])
        assert B.g2_compress(B.G2C.mul(B.hash_to_g2(msg, v["dst"].encode()), sk)).hex() == v["sig"]


def test_generators():
    g = load("kat.json")["generators"]
    assert B.g1_compress(B.G1_GEN).hex() == g["g1"]
    assert B.g2_compress(B.G2_GEN).hex() == g["g2"]
    assert twin.g1_mul_gen(1).hex() == g["g1"]


def test_beacon_message_kat():
    for v in load("kat.json")["beacon_message"]:
        m = T.beacon_message(hx(v["prev_sig"]), v["prev_round"], v["round"])
        assert m.hex() == v["expected"]
        assert twin.beacon_message(hx(v["prev_sig"]), v["prev_round"], v["round"]).hex() == v["expected"]


def test_reference_g1_keys_decode():
    keys = load("reference_g1_keys.json")["keys"]
    assert len(keys) >= 15
    for k in keys:
        b = hx(k["key"])
        assert B.g1_compress(B.g1_decompress(b)) == b


def test_hash_to_g2_drand_dst_twin_matches_pyref_fixture():
    v = load("hash_to_g2_nul.json")
    for x in v["vectors"]:
        assert twin.hash_to_g2(hx(x["msg"]), v["dst"].encode()).hex() == x["h"]
    x = v["vectors"][0]
    assert B.g2_compress(B.hash_to_g2(hx(x["msg"]), v["dst"].encode())).hex() == x["h"]


def test_chain_fixture_consistent():
    c = chain()
    pk = hx(c["pk"])
    prev = hx(c["genesis_seed"])
    for r in c["rounds"]:
        assert hashlib.sha256(r["prev_round"].to_bytes(8, "big") + prev + r["round"].to_bytes(8, "big")).hexdigest() == r["msg"]
        assert hashlib.sha256(hx(r["sig"])).hexdigest() == r["randomness"]
        prev = hx(r["sig"])
    _, _, _, sigs, msgs = chain_arrays(c)
    st = twin.verify_batch(pk, msgs, sigs, threads=4)
    assert list(st) == [0] * len(c["rounds"])
    # wrong round -> invalid
    assert twin.verify(pk, hx(c["rounds"][1]["msg"]), hx(c["rounds"][0]["sig"])) == 1


def test_chain_recover_fixture():
    c = chain()
    commits = [hx(x) for x in c["commits"]]
    for pr, rd in zip(c["partial_rounds"], c["rounds"]):
        parts = [hx(p) for p in pr["partials"]]
        sig, rs, ss = twin.recover(commits, hx(rd["msg"]), parts, c["t"], c["n"])
        assert rs == 0 and sig.hex() == rd["sig"]
        assert ss[:3] == [0, 0, 0] and ss[3:] == [255, 255]


def test_adversarial_fixture_twin():
    a = load("adversarial_t3n5.json")
    commits = [hx(x) for x in a["commits"]]
    for case in a["cases"]:
        msg = hx(case["msg"])
        parts = [hx(p) for p in case["partials"]]
        assert [twin.verify_partial(commits, msg, p) for p in parts] == case["verify_status"]
        sig, rs, ss = twin.recover(commits, msg, parts, a["t"], a["n"])
        assert rs == case["recover_status"]
        assert ss == case["share_status"]
        if rs == 0:
            assert sig.hex() == case["recover_sig"]


def test_adversarial_fixture_pyref_sample():
    a = load("adversarial_t3n5.json")
    commits = [hx(x) for x in a["commits"]]
    case = a["cases"][0]
    msg = hx(case["msg"])
    parts = [hx(p) for p in case["partials"]]
    got = [T.verify_partial_status(commits, msg, p) for p in parts[:3]]
    assert got == case["verify_status"][:3]


def test_g2_decode_edges():
    for case in load("g2_decode_edges.json")["cases"]:
        b = hx(case["enc"])
        try:
            B.g2_decompress(b)
            ok = True
        except B.DecodeError:
            ok = False
        assert ok == case["decodes"], case["name"]


def test_lagrange_pyref():
    # interpolation of a known polynomial at 0 from any t points
    coeffs = [5, 7, 11]
    pts = [(i, sum(c * (i + 1) ** j for j, c in enumerate(coeffs)) % B.R) for i in (4, 1, 9)]
    lam = T.lagrange_at_zero([i for i, _ in pts])
    assert sum(l * y for l, (_, y) in zip(lam, pts)) % B.R == coeffs[0]


@pytest.mark.parametrize("idx", [0, 3, 64])
def test_pubpoly_eval_twin_vs_pyref(idx):
    c = chain()
    commits = [hx(x) for x in c["commits"]]
    st, out = twin.pubpoly_eval(commits, idx)
    assert st == 0
    assert B.g1_compress(T.pubpoly_eval(commits, idx)) == out


def test_group_pk_constant():
    from tools import synthetic as S

    assert twin.g1_mul_gen(S.master_secret()) == S.GROUP_PK == hx(chain()["pk"])
    assert B.g1_compress(B.G1C.mul(B.G1_GEN, S.master_secret())) == S.GROUP_PK


def test_chain_file_prefix_matches_fixture():
    """data/chain_v1_*.bin (generated by tools/gen_chain.py, shipped to the GPU box) starts with the fixture."""
    import glob

    import numpy as np

    files = glob.glob(os.path.join(ROOT, "data", "chain_v1_*.bin"))
    if not files:
        pytest.skip("no chain file generated here")
    c = chain()
    mm = np.memmap(files[0], dtype=np.uint8, mode="r")
    for k, r in enumerate(c["rounds"]):
        assert bytes(mm[96 * k:96 * k + 96]).hex() == r["sig"]


def test_group_commits_fixture():
    from tools import synthetic as S

    g = load("groups.json")
    for t in (3, 33, 129):
        coeffs = S.poly_coeffs(t)
        assert g["t%d" % t][0] == S.GROUP_PK.hex()
        for j in (1, t - 1):
            assert twin.g1_mul_gen(coeffs[j]).hex() == g["t%d" % t][j]
    assert g["t3"] == chain()["commits"]


def test_torsion_fixture_decodes_outside_g2():
    """tests/golden/g2_torsion.json: on the curve (decodes without the subgroup check), outside G2, and
    the twin's bls.Verify rejects each as a decode error."""
    from oracle.pyref import bls12381 as B
    from tests.fixtures import chain, hx, load

    c = chain()
    pk = hx(c["pk"])
    for case in load("g2_torsion.json")["cases"]:
        pt = B.g2_decompress(hx(case["sig"]), subgroup_check=False)
        assert B.G2C.on_curve(pt) and not B.g2_in_subgroup(pt)
        msg = hx(c["rounds"][case["round_index"]]["msg"])
        assert twin.verify(pk, msg, hx(case["sig"])) == 2


def _ref_points():
    t = load("reference_test_json_points.json")
    return [hx(p["hex"]) for p in t["points"]]  # Public (G2), Previous (G1), Signature (G1)


def _g2_variants(pub):
    """Public's c0 <-> c1 swap (flags kept on the first half), the compression flag cleared, the infinity flag set
    with a non-zero body, the sign flag flipped (the negated point: still valid)."""
    swapped = bytes([pub[48] | (pub[0] & 0xE0)]) + pub[49:96] + bytes([pub[0] & 0x1F]) + pub[1:48]
    return {"swapped": swapped, "uncompressed_flag": bytes([pub[0] & 0x7F]) + pub[1:],
            "infinity_flag": bytes([pub[0] | 0x40]) + pub[1:], "sign_flipped": bytes([pub[0] ^ 0x20]) + pub[1:]}


def test_reference_test_json_points_decode():
    """The reference's only G2 encoding (test/test-integration/test.json:5, `Public` = x g2) and its two G1 signatures
    (`Previous`, `Signature`; json_output.go:22,27) decode in pyref (on the curve, in the subgroup) and re-encode byte
    for byte; the twin decodes them too: as (key, sigma) of a bls.Verify they give a pairing failure (status 1), not a
    decode error (2, 4).  Swapping Public's c0 and c1 halves, clearing its compression flag or setting its infinity
    flag makes it undecodable for both (status 2); flipping its sign flag gives the valid negated point (status 1).
    This pins G2 decompression's c1 || c0 order and flag handling to data the reference holds."""
    pub, prev, sig = _ref_points()
    assert B.g2_compress(B.g2_decompress(pub)) == pub
    for g1 in (prev, sig):
        assert B.g1_compress(B.g1_decompress(g1)) == g1
    msg = hashlib.sha256(b"test.json").digest()
    for g1 in (prev, sig):
        assert twin.verify(g1, msg, pub) == 1
    want = {"swapped": 2, "uncompressed_flag": 2, "infinity_flag": 2, "sign_flipped": 1}
    for name, v in _g2_variants(pub).items():
        assert twin.verify(sig, msg, v) == want[name], name
        try:
            B.g2_decompress(v)
            py = 1
        except B.DecodeError:
            py = 2
        assert py == want[name], name
