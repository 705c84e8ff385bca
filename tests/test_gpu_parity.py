"""Parity of the HIP path (through the C-ABI) with the oracle: committed golden fixtures, the CPU twin on
the same seeded inputs, and size-independent properties at larger sizes.  Bit-exact throughout."""
import hashlib

import numpy as np
import pytest

from drand_amd import _lib as L
from drand_amd import tbls
from oracle import twin
from oracle.pyref import tbls as T
from tests.fixtures import chain, chain_arrays, group, hx, load
from tools import corrupt as C
from tools import synthetic as S

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def device():
    L.lib(0)
    yield


def test_hash_to_g2_golden():
    v = load("hash_to_g2_nul.json")
    out = tbls.hash_to_g2([hx(x["msg"]) for x in v["vectors"]])
    assert [bytes(o).hex() for o in out] == [x["h"] for x in v["vectors"]]


def test_hash_to_g2_rfc9380_empty_msg():
    for x in load("kat.json")["hash_to_g2_rfc9380"]:
        out = tbls.hash_to_g2([x["msg"].encode()], dst=x["dst"].encode())
        assert bytes(out[0]).hex() == x["compressed"]


def test_hash_to_g2_odd_lengths_vs_twin():
    for ln in (0, 1, 55, 56, 64, 100, 200):
        msgs = [hashlib.sha256(b"m%d/%d" % (ln, i)).digest() * 8 for i in range(3)]
        msgs = [m[:ln] for m in msgs]
        out = tbls.hash_to_g2(msgs)
        for i, m in enumerate(msgs):
            assert bytes(out[i]) == twin.hash_to_g2(m), (ln, i)


def test_beacon_messages_randomness_links_golden():
    c = chain()
    pr, rr, ps, sigs, msgs = chain_arrays(c)
    assert np.array_equal(tbls.beacon_messages(pr, rr, ps), msgs)
    rnd = tbls.randomness(sigs)
    assert [bytes(x).hex() for x in rnd] == [r["randomness"] for r in c["rounds"]]
    links = tbls.check_links(0, hx(c["genesis_seed"]), pr, rr, ps, sigs)
    assert list(links) == [0] * len(rr)
    ps2 = list(ps)
    ps2[10] = bytes(96)
    rr2 = list(rr)
    rr2[20] = rr2[19]
    links = tbls.check_links(0, hx(c["genesis_seed"]), pr, rr2, ps2, sigs)
    want = T.check_links(0, hx(c["genesis_seed"]), pr, rr2, ps2, [bytes(s) for s in sigs])
    assert links.tolist() == want
    assert np.nonzero(links)[0].tolist() == [10, 20, 21]  # 21: its prev_round no longer matches round 20


def test_verify_beacons_golden_chain():
    c = chain()
    pr, rr, ps, sigs, msgs = chain_arrays(c)
    st = tbls.verify_beacons(hx(c["pk"]), pr, rr, ps, sigs, seed=3)
    assert list(st) == [0] * len(rr)


def _corrupt_sigs(sigs):
    bad = sigs.copy()
    bad[1] = sigs[2]                       # valid signature, wrong round -> 1
    bad[5, 40] ^= 0x04                     # x bit flip -> decode error (off curve) or invalid
    bad[9] = 0
    bad[9, 0] = 0xC0                       # infinity -> 1
    bad[13] = np.frombuffer(hashlib.sha256(b"x").digest() * 3, np.uint8)  # random -> 2
    bad[17, 0] &= 0x7F                     # uncompressed flag cleared -> 2
    bad[21, 0] ^= 0x20                     # sign flag flipped -> -sigma -> 1
    bad[25, 47] ^= 1                       # low bit of x.c1
    bad[30, 0] |= 0x1F                     # x >= p -> 2
    return bad


def test_verify_beacons_corrupted_matches_twin():
    c = chain()
    pr, rr, ps, sigs, msgs = chain_arrays(c)
    bad = _corrupt_sigs(sigs)
    pk = hx(c["pk"])
    st = tbls.verify_beacons(pk, pr, rr, ps, bad, seed=11)
    want = [twin.verify(pk, bytes(msgs[i]), bytes(bad[i])) for i in range(len(rr))]
    assert list(st) == want
    assert sum(1 for w in want if w) >= 8


def test_verify_wrong_and_bad_keys():
    c = chain()
    _, _, _, sigs, msgs = chain_arrays(c)
    other = twin.g1_mul_gen(12345)
    st = tbls.verify_recovered_batch(other, msgs[:8], sigs[:8], seed=5)
    assert list(st) == [1] * 8
    bad_pk = bytearray(hx(c["pk"]))
    bad_pk[0] &= 0x7F
    st = tbls.verify_recovered_batch(bytes(bad_pk), msgs[:8], sigs[:8], seed=5)
    assert list(st) == [4] * 8


def test_verify_seed_independence():
    c = chain()
    pr, rr, ps, sigs, msgs = chain_arrays(c)
    bad = _corrupt_sigs(sigs)
    pk = hx(c["pk"])
    a = tbls.verify_beacons(pk, pr, rr, ps, bad, seed=1)
    b = tbls.verify_beacons(pk, pr, rr, ps, bad, seed=0)  # seed from the OS
    assert np.array_equal(a, b)


def test_sign_matches_twin_and_fixture():
    c = chain()
    rd = c["partial_rounds"][0]
    msg = hx(c["rounds"][0]["msg"])
    coeffs = [int(x, 16) for x in c["coeffs"]]
    shares = [(i, S.share_value(coeffs, i)) for i in range(c["n"])]
    out = tbls.sign_batch([v for _, v in shares], [msg] * c["n"], [i for i, _ in shares])
    assert [bytes(o).hex() for o in out] == rd["partials"]
    out = tbls.sign_batch([coeffs[0]], [msg])
    assert bytes(out[0]).hex() == c["rounds"][0]["sig"]


def test_pubpoly_eval_vs_twin():
    c = chain()
    commits = [hx(x) for x in c["commits"]]
    pub = tbls.PubPoly(commits)
    idx = [0, 1, 2, 3, 4, 63, 255, 65535]
    out = tbls.pubpoly_eval(pub, idx)
    for i, o in zip(idx, out):
        assert o == twin.pubpoly_eval(commits, i)[1]


def test_verify_partials_and_recover_golden():
    c = chain()
    pub = tbls.PubPoly([hx(x) for x in c["commits"]])
    prs = c["partial_rounds"]
    msgs = [hx(c["rounds"][k]["msg"]) for k in range(len(prs))]
    parts = np.array([[list(hx(p)) for p in pr["partials"]] for pr in prs], np.uint8)
    st = tbls.verify_partial_batch(pub, msgs, parts, seed=2)
    assert st.tolist() == [[0] * 5] * len(prs)
    sigs, rs, ss = tbls.recover_batch(pub, msgs, parts, c["t"], c["n"], seed=2)
    assert rs.tolist() == [0] * len(prs)
    assert [bytes(s).hex() for s in sigs] == [c["rounds"][k]["sig"] for k in range(len(prs))]
    assert ss.tolist() == [[0, 0, 0, 255, 255]] * len(prs)


def test_adversarial_golden():
    a = load("adversarial_t3n5.json")
    pub = tbls.PubPoly([hx(x) for x in a["commits"]])
    for case in a["cases"]:
        parts = np.array([list(hx(p)) for p in case["partials"]], np.uint8)[None]
        msg = [hx(case["msg"])]
        st = tbls.verify_partial_batch(pub, msg, parts, seed=4)
        assert st[0].tolist() == case["verify_status"], case["modes"]
        sigs, rs, ss = tbls.recover_batch(pub, msg, parts, a["t"], a["n"], seed=4)
        assert int(rs[0]) == case["recover_status"], case["modes"]
        assert ss[0].tolist() == case["share_status"], case["modes"]
        if case["recover_status"] == 0:
            assert bytes(sigs[0]).hex() == case["recover_sig"]


def test_scheme_api_errors():
    c = chain()
    pub = tbls.PubPoly([hx(x) for x in c["commits"]])
    rd = c["rounds"][0]
    p0 = hx(c["partial_rounds"][0]["partials"][0])
    sch = tbls.Scheme
    assert sch.index_of(p0) == 0
    sch.verify_partial(pub, hx(rd["msg"]), p0)
    sch.verify_recovered(pub.commit(), hx(rd["msg"]), hx(rd["sig"]))
    with pytest.raises(tbls.SchemeError):
        sch.verify_recovered(pub.commit(), hx(c["rounds"][1]["msg"]), hx(rd["sig"]))
    with pytest.raises(tbls.SchemeError):
        sch.verify_partial(pub, hx(c["rounds"][1]["msg"]), p0)
    with pytest.raises(tbls.SchemeError):
        sch.index_of(b"\x00")
    parts = [hx(p) for p in c["partial_rounds"][0]["partials"]]
    assert sch.recover(pub, hx(rd["msg"]), parts[2:], 3, 5).hex() == rd["sig"]
    with pytest.raises(tbls.SchemeError):
        sch.recover(pub, hx(rd["msg"]), parts[3:], 3, 5)


def _group_rounds(t, n, R, frac, label):
    coeffs, commits, shares = group(t, n)
    msgs = [hashlib.sha256(b"%s/%d" % (label, r)).digest() for r in range(R)]
    sc = [v for _ in range(R) for _, v in shares]
    idx = [i for _ in range(R) for i, _ in shares]
    mm = [m for m in msgs for _ in range(n)]
    parts = tbls.sign_batch(sc, mm, idx).reshape(R, n, 98)

    def resign(reqs):
        sc2 = [(shares[i][1] + ds) % S.R for (r, i, ds, dr) in reqs]
        m2 = [msgs[(r + dr) % R] if dr else msgs[r] for (r, i, ds, dr) in reqs]
        return tbls.sign_batch(sc2, m2)

    items = C.pick(R, n, frac, seed=label)
    C.corrupt_batch(parts, items, n, resign)
    return coeffs, commits, msgs, parts, items


@pytest.mark.parametrize("t,n,R", [(33, 64, 4), (129, 256, 1)])
def test_large_group_corrupted_vs_twin(t, n, R):
    coeffs, commits, msgs, parts, items = _group_rounds(t, n, R, 0.1, b"lg%d" % n)
    pub = tbls.PubPoly(commits)
    st = tbls.verify_partial_batch(pub, msgs, parts, seed=9)
    want = np.array([[twin.verify_partial(commits, msgs[r], bytes(parts[r, j])) for j in range(n)] for r in range(R)])
    assert np.array_equal(st, want)
    assert (want != 0).sum() >= len(items) // 2
    sigs, rs, ss = tbls.recover_batch(pub, msgs, parts, t, n, seed=9)
    tw_sigs, tw_rs, tw_ss = twin.recover_batch(commits, t, n, np.array([list(m) for m in msgs], np.uint8), parts, 8)
    assert np.array_equal(rs, tw_rs) and np.array_equal(ss, tw_ss)
    assert np.array_equal(sigs[rs == 0], tw_sigs[tw_rs == 0])
    x = coeffs[0]
    for r in range(R):
        if rs[r] == 0:
            assert bytes(sigs[r]) == twin.sign(x, msgs[r])


@pytest.mark.parametrize("t,n,R,frac", [(33, 64, 64, 0.1), (129, 256, 24, 0.1), (129, 256, 8, 0.3)])
def test_recover_corrupted_at_scale_vs_twin(t, n, R, frac):
    """C3 / C5 shapes over many rounds (the group tests, the speculative passes and the final exact pass of
    the per-item check): signatures, round statuses and every share status equal the CPU twin's Recover
    (kyber's algorithm: each examined share verified in input order)."""
    coeffs, commits, msgs, parts, items = _group_rounds(t, n, R, frac, b"rs%d/%d" % (n, R))
    pub = tbls.PubPoly(commits)
    sigs, rs, ss = tbls.recover_batch(pub, msgs, parts, t, n, seed=31)
    tw_sigs, tw_rs, tw_ss = twin.recover_batch(commits, t, n, np.array([list(m) for m in msgs], np.uint8), parts, 16)
    assert np.array_equal(rs, tw_rs) and np.array_equal(ss, tw_ss)
    assert np.array_equal(sigs[rs == 0], tw_sigs[tw_rs == 0])
    assert (ss == L.ST_BAD_SIG).sum() > 0


def test_not_enough_shares_many_rounds():
    t, n, R = 3, 5, 6
    coeffs, commits, msgs, parts, _ = _group_rounds(t, n, R, 0.0, b"ne")
    parts[2, :3, 50] ^= 0x01   # 3 of 5 broken in round 2 -> not enough
    parts[4, 1] = parts[4, 0]  # duplicate index in round 4 among the first t collected
    pub = tbls.PubPoly(commits)
    sigs, rs, ss = tbls.recover_batch(pub, msgs, parts, t, n, seed=8)
    tw = [twin.recover(commits, msgs[r], [bytes(p) for p in parts[r]], t, n) for r in range(R)]
    assert rs.tolist() == [w[1] for w in tw]
    assert ss.tolist() == [w[2] for w in tw]
    assert rs[2] == L.ST_NOT_ENOUGH and rs[4] == L.ST_NOT_ENOUGH


def test_verify_at_size_exact_bitmap():
    """2048 independent rounds signed on the GPU: all valid, then 1% flipped at known positions."""
    R = 2048
    x = S.master_secret()
    pk = twin.g1_mul_gen(x)
    msgs = np.frombuffer(b"".join(hashlib.sha256(b"sz/%d" % r).digest() for r in range(R)), np.uint8).reshape(R, 32)
    sigs = tbls.sign_batch([x] * R, msgs)
    st = tbls.verify_recovered_batch(pk, msgs, sigs, seed=21)
    assert not st.any()
    bad_pos = sorted({(r * 7919) % R for r in range(R // 100)})
    bad = sigs.copy()
    for p in bad_pos:
        bad[p] = sigs[(p + 1) % R]
    st = tbls.verify_recovered_batch(pk, msgs, bad, seed=22)
    assert np.nonzero(st)[0].tolist() == bad_pos
    assert set(st[bad_pos].tolist()) == {L.ST_BAD_SIG}


def test_valid_batches_pass_on_the_batch_path_many_seeds():
    """The RLC batch equation (MSM, cooperative Miller loops, final exponentiation) must accept valid
    batches for every seed: the per-item fallback would hide a wrong batch path behind correct verdicts."""
    c = chain()
    pr, rr, ps, sigs, msgs = chain_arrays(c)
    pk = hx(c["pk"])
    bad_seeds = []
    for seed in range(1, 121):
        st = tbls.verify_beacons(pk, pr, rr, ps, sigs, seed=seed)
        ok, iso = L.last_batch_flags()
        assert not st.any()
        if not ok or iso:
            bad_seeds.append(seed)
    assert bad_seeds == []


def test_valid_partial_batches_pass_on_the_batch_path():
    c = chain()
    pub = tbls.PubPoly([hx(x) for x in c["commits"]])
    prs = c["partial_rounds"]
    msgs = [hx(c["rounds"][k]["msg"]) for k in range(len(prs))]
    parts = np.array([[list(hx(p)) for p in pr["partials"]] for pr in prs], np.uint8)
    for seed in range(1, 41):
        st = tbls.verify_partial_batch(pub, msgs, parts, seed=seed)
        assert not st.any()
        assert L.last_batch_flags() == (True, False), seed


def test_torsion_signatures_rejected_like_the_twin():
    """On-curve signatures outside G2 (sigma + E with E of order 13, 23, 299; uncleared hash outputs,
    tests/golden/g2_torsion.json): the beacon path decodes without a per-item subgroup check and batches
    it on the MSM window sums (msm.h), so each such item must still end as a decode error (status 2),
    alone in an otherwise valid chain and all together, for many seeds, exactly as the twin's per-item
    bls.Verify (decode with subgroup check) says."""
    c = chain()
    pr, rr, ps, sigs, msgs = chain_arrays(c)
    pk = hx(c["pk"])
    cases = load("g2_torsion.json")["cases"]
    for case in cases:
        i = case["round_index"]
        bad = sigs.copy()
        bad[i] = np.frombuffer(hx(case["sig"]), np.uint8)
        assert twin.verify(pk, bytes(msgs[i]), bytes(bad[i])) == L.ST_SIG_DECODE
        for seed in (3, 4, 5):
            st = tbls.verify_beacons(pk, pr, rr, ps, bad, seed=seed)
            assert np.nonzero(st)[0].tolist() == [i], (case["kind"], seed)
            assert st[i] == L.ST_SIG_DECODE
            assert L.last_batch_flags()[0] is False  # the batch check caught it
    bad = sigs.copy()
    idx = [case["round_index"] for case in cases]
    for case in cases:
        bad[case["round_index"]] = np.frombuffer(hx(case["sig"]), np.uint8)
    bad[7] = sigs[8]  # plus a wrong-round signature (pairing failure)
    want = [twin.verify(pk, bytes(msgs[j]), bytes(bad[j])) for j in range(len(rr))]
    for seed in range(20, 30):
        st = tbls.verify_beacons(pk, pr, rr, ps, bad, seed=seed)
        assert list(st) == want
    assert sorted(np.nonzero(want)[0].tolist()) == sorted(idx + [7])


def test_torsion_signature_in_a_large_batch():
    """One valid signature plus a torsion point E (ord 13) among 4096 GPU-signed valid rounds: exactly
    that item is rejected, as a decode error."""
    from oracle.pyref import bls12381 as B

    R = 4096
    x = S.master_secret()
    pk = twin.g1_mul_gen(x)
    case = load("g2_torsion.json")["cases"][0]
    j = case["round_index"]
    e = B.G2C.add(B.g2_decompress(hx(case["sig"]), subgroup_check=False),
                  B.G2C.neg(B.g2_decompress(hx(chain()["rounds"][j]["sig"]))))
    msgs = np.frombuffer(b"".join(hashlib.sha256(b"tor/%d" % r).digest() for r in range(R)), np.uint8).reshape(R, 32)
    sigs = tbls.sign_batch([x] * R, msgs)
    st = tbls.verify_recovered_batch(pk, msgs, sigs, seed=31)
    assert not st.any() and L.last_batch_flags() == (True, False)
    bad = B.g2_compress(B.G2C.add(B.g2_decompress(bytes(sigs[1234])), e))
    assert twin.verify(pk, bytes(msgs[1234]), bad) == L.ST_SIG_DECODE
    sigs[1234] = np.frombuffer(bad, np.uint8)
    st = tbls.verify_recovered_batch(pk, msgs, sigs, seed=32)
    assert np.nonzero(st)[0].tolist() == [1234] and st[1234] == L.ST_SIG_DECODE
