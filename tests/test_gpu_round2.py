"""Round-2 parity tests of the HIP path through the C-ABI: the reference's own fixtures through the kernels,
the runtime DST switch, the live-round Recover with known verdicts, the bound on key slots, the batch-bound
RLC coefficients and the sharded 1M-round chain (BASELINE configs[3]).  Bit-exact throughout."""
import hashlib
import os

import numpy as np
import pytest

from drand_amd import _lib as L
from drand_amd import tbls
from oracle import twin
from oracle.pyref import bls12381 as B
from tests.fixtures import chain, chain_arrays, group, hx, load
from tools import corrupt as C
from tools import synthetic as S

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module", autouse=True)
def device():
    L.lib(0)
    yield
    tbls.set_hash_dst(None)
    twin.set_dst(None)


def test_reference_g1_keys_through_the_kernels():
    """The reference's own 25 G1 keys (deploy/200409/group.toml, demo/docker/data/*): k_decode_g1 decodes each
    (flags, canonical x, curve, subgroup) and PubPoly.Eval with t = 1 returns the constant term, which
    k_pubpoly_eval compresses back to the input bytes."""
    keys = [hx(k["key"]) for k in load("reference_g1_keys.json")["keys"]]
    assert len(keys) == 25
    for k in keys:
        out = tbls.pubpoly_eval(tbls.PubPoly([k]), [0, 1, 65535])
        assert out == [k, k, k]


def test_g2_decode_edges_through_verify():
    """tests/golden/g2_decode_edges.json through dg_verify: every encoding that must not decode gets status 2
    (sigma decode), exactly as the CPU twin's bls.Verify says, inside one batch with valid rounds."""
    c = chain()
    _, _, _, sigs, msgs = chain_arrays(c)
    pk = hx(c["pk"])
    cases = load("g2_decode_edges.json")["cases"]
    n = len(cases)
    s = sigs[:n].copy()
    for i, case in enumerate(cases):
        s[i] = np.frombuffer(hx(case["enc"]), np.uint8)
    st = tbls.verify_recovered_batch(pk, msgs[:n], s, seed=3)
    want = [twin.verify(pk, bytes(msgs[i]), bytes(s[i])) for i in range(n)]
    assert st.tolist() == want
    for i, case in enumerate(cases):
        if not case["decodes"]:
            assert st[i] == L.ST_SIG_DECODE, case["name"]


def test_hash_dst_switch_everywhere():
    """dg_set_hash_dst changes the hash of sign, verify, VerifyPartial and Recover at run time: with another
    DST the library and the twin (set to the same DST) agree bit for bit, signatures made under one DST fail
    under the other, and restoring the default restores the golden chain."""
    c = chain()
    pr, rr, ps, sigs, msgs = chain_arrays(c)
    pk = hx(c["pk"])
    x = int(c["coeffs"][0], 16)
    other = b"BLS_SIG_BLS12381G2_XMD:SHA-256_SSWU_RO_POP_"
    assert tbls.hash_dst() == L.DST_NUL
    try:
        tbls.set_hash_dst(other)
        twin.set_dst(other)
        assert tbls.hash_dst() == other
        s2 = tbls.sign_batch([x] * 8, msgs[:8])
        for i in range(8):
            assert bytes(s2[i]) == twin.sign(x, bytes(msgs[i])) != bytes(sigs[i])
        assert tbls.verify_recovered_batch(pk, msgs[:8], s2, seed=4).tolist() == [0] * 8
        assert tbls.verify_recovered_batch(pk, msgs[:8], sigs[:8], seed=4).tolist() == [1] * 8
        st = tbls.verify_beacons(pk, pr[:8], rr[:8], ps[:8], sigs[:8], seed=5)
        assert st.tolist() == [1] * 8
        # threshold path under the other DST
        coeffs = [int(h, 16) for h in c["coeffs"]]
        pub = tbls.PubPoly([hx(h) for h in c["commits"]])
        shares = [S.share_value(coeffs, i) for i in range(5)]
        parts = tbls.sign_batch(shares * 2, [bytes(msgs[0])] * 5 + [bytes(msgs[1])] * 5, list(range(5)) * 2)
        parts = parts.reshape(2, 5, 98)
        assert not tbls.verify_partial_batch(pub, msgs[:2], parts, seed=6).any()
        rs_sigs, rs, _ = tbls.recover_batch(pub, msgs[:2], parts, 3, 5, seed=6)
        assert not rs.any() and [bytes(v) for v in rs_sigs] == [bytes(s2[0]), bytes(s2[1])]
        w = twin.recover([hx(h) for h in c["commits"]], bytes(msgs[0]), [bytes(p) for p in parts[0]], 3, 5)
        assert w[0] == bytes(s2[0])
    finally:
        tbls.set_hash_dst(None)
        twin.set_dst(None)
    assert tbls.hash_dst() == L.DST_NUL
    assert not tbls.verify_beacons(pk, pr, rr, ps, sigs, seed=7).any()


def _group_rounds(t, n, R, frac, label):
    coeffs, commits, shares = group(t, n)
    msgs = [hashlib.sha256(b"%s/%d" % (label, r)).digest() for r in range(R)]
    parts = tbls.sign_batch([v for _ in range(R) for _, v in shares], [m for m in msgs for _ in range(n)],
                            [i for _ in range(R) for i, _ in shares]).reshape(R, n, 98)

    def resign(reqs):
        sc2 = [(shares[i][1] + ds) % S.R for (r, i, ds, dr) in reqs]
        m2 = [msgs[(r + dr) % R] if dr else msgs[r] for (r, i, ds, dr) in reqs]
        return tbls.sign_batch(sc2, m2)

    items = C.pick(R, n, frac, seed=label)
    C.corrupt_batch(parts, items, n, resign)
    return coeffs, commits, msgs, parts


@pytest.mark.parametrize("t,n,R", [(3, 5, 16), (33, 64, 6)])
def test_recover_verified_equals_recover(t, n, R):
    """The live-round Recover (dg_recover_verified) fed ProcessBeacon's VerifyPartial verdicts gives exactly
    dg_recover's signatures, round statuses and share statuses (and the twin's), without re-verifying."""
    coeffs, commits, msgs, parts = _group_rounds(t, n, R, 0.3, b"rv%d" % n)
    pub = tbls.PubPoly(commits)
    vst = tbls.verify_partial_batch(pub, msgs, parts, seed=12)
    a = tbls.recover_batch(pub, msgs, parts, t, n, seed=12)
    b = tbls.recover_verified_batch(pub, msgs, parts, vst, t, n)
    for x, y in zip(a, b):
        assert np.array_equal(x, y)
    tw = twin.recover_batch(commits, t, n, np.array([list(m) for m in msgs], np.uint8), parts, 8)
    assert np.array_equal(b[1], tw[1]) and np.array_equal(b[2], tw[2])
    assert np.array_equal(b[0][b[1] == 0], tw[0][tw[1] == 0])


def test_recover_verified_trusts_only_ok_verdicts():
    """A valid partial whose verdict is not OK is skipped (as Recover skips a failing share)."""
    coeffs, commits, msgs, parts = _group_rounds(3, 5, 2, 0.0, b"rvt")
    pub = tbls.PubPoly(commits)
    vst = np.zeros((2, 5), np.uint8)
    vst[0, :3] = L.ST_BAD_SIG       # round 0: only 2 OK -> not enough
    vst[1, 0] = L.ST_SIG_DECODE     # round 1: shares 1, 2, 3 collected
    sigs, rs, ss = tbls.recover_verified_batch(pub, msgs, parts, vst, 3, 5)
    assert rs.tolist() == [L.ST_NOT_ENOUGH, 0]
    assert ss.tolist() == [[1, 1, 1, 0, 0], [2, 0, 0, 0, 255]]
    assert bytes(sigs[1]) == twin.sign(coeffs[0], msgs[1])


def test_fresh_index_every_round_is_bounded_and_exact():
    """A signer that uses a different share index in every round (ADVICE: each distinct index used to become
    a key set of its own): those indices stay out of the batch equation and are checked alone; statuses and
    Recover outputs equal the twin's."""
    t, n, R = 3, 5, 48
    coeffs, commits, shares = group(t, n)
    msgs = [hashlib.sha256(b"fresh/%d" % r).digest() for r in range(R)]
    k = n + 1
    idx = [[i for i in range(n)] + [100 + r] for r in range(R)]
    sc = [S.share_value(coeffs, i) for r in range(R) for i in idx[r]]
    parts = tbls.sign_batch(sc, [m for m in msgs for _ in range(k)], [i for r in range(R) for i in idx[r]])
    parts = parts.reshape(R, k, 98)
    parts[5, 5, 60] ^= 1  # one broken fresh-index share
    # put the fresh share first in some rounds, so Recover examines it
    for r in range(0, R, 3):
        parts[r] = parts[r][[5, 0, 1, 2, 3, 4]]
    pub = tbls.PubPoly(commits)
    st = tbls.verify_partial_batch(pub, msgs, parts, seed=13)
    want = np.array([[twin.verify_partial(commits, msgs[r], bytes(parts[r, j])) for j in range(k)] for r in range(R)])
    assert np.array_equal(st, want) and want[5, :5].tolist() == [0] * 5 and want[5, 5] != 0
    ok, iso = L.last_batch_flags()
    assert ok and iso  # the batch equation held for the frequent indices; the fresh ones were checked alone
    sigs, rs, ss = tbls.recover_batch(pub, msgs, parts, t, n, seed=13)
    tw = twin.recover_batch(commits, t, n, np.array([list(m) for m in msgs], np.uint8), parts, 8)
    assert np.array_equal(rs, tw[1]) and np.array_equal(ss, tw[2]) and np.array_equal(sigs, tw[0])


def _old_alpha(seed, r):
    """The round-1 coefficient alpha_r = SHA-256(BE64 seed || BE64 r)[0..8) | 1, a function of the seed alone."""
    d = hashlib.sha256(seed.to_bytes(8, "big") + r.to_bytes(8, "big")).digest()
    return int.from_bytes(d[:8], "big") | 1


def test_known_seed_cannot_cancel_errors():
    """Two invalid signatures crafted so their errors cancel in sum_r alpha_r sigma_r for the coefficients a
    known seed used to fix (sigma'_1 = sigma_1 + alpha_2 E, sigma'_2 = sigma_2 - alpha_1 E, E in G2): the
    coefficients are now bound to the batch contents, so the batch equation fails and both items are
    rejected one by one, as the twin rejects them."""
    c = chain()
    _, _, _, sigs, msgs = chain_arrays(c)
    pk = hx(c["pk"])
    seed = 0x1234
    r1, r2 = 3, 11
    E = B.G2C.mul(B.G2_GEN, 987654321)
    a1, a2 = _old_alpha(seed, r1), _old_alpha(seed, r2)
    bad = sigs.copy()
    s1 = B.G2C.add(B.g2_decompress(bytes(sigs[r1])), B.G2C.mul(E, a2))
    s2 = B.G2C.add(B.g2_decompress(bytes(sigs[r2])), B.G2C.neg(B.G2C.mul(E, a1)))
    bad[r1] = np.frombuffer(B.g2_compress(s1), np.uint8)
    bad[r2] = np.frombuffer(B.g2_compress(s2), np.uint8)
    # the crafted pair does cancel for the seed-only coefficients
    lhs = B.G2C.add(B.G2C.mul(s1, a1), B.G2C.mul(s2, a2))
    rhs = B.G2C.add(B.G2C.mul(B.g2_decompress(bytes(sigs[r1])), a1), B.G2C.mul(B.g2_decompress(bytes(sigs[r2])), a2))
    assert B.G2C.eq(lhs, rhs)
    st = tbls.verify_recovered_batch(pk, msgs, bad, seed=seed)
    want = [twin.verify(pk, bytes(msgs[i]), bytes(bad[i])) for i in range(len(msgs))]
    assert st.tolist() == want and np.nonzero(st)[0].tolist() == [r1, r2]
    assert L.last_batch_flags()[0] is False


def test_batch_coefficients_depend_on_contents():
    """Same seed, valid batches that differ in one item: both pass on the batch path (and a valid batch passes
    for every seed: tests/test_gpu_parity.py)."""
    c = chain()
    pr, rr, ps, sigs, msgs = chain_arrays(c)
    pk = hx(c["pk"])
    assert not tbls.verify_beacons(pk, pr, rr, ps, sigs, seed=99).any() and L.last_batch_flags() == (True, False)
    assert not tbls.verify_beacons(pk, pr[:-1], rr[:-1], ps[:-1], sigs[:-1], seed=99).any()
    assert L.last_batch_flags() == (True, False)


def _chain_file(n):
    """The digest-pinned chain file of n rounds (tools/synthetic.find_chain); a missing or altered file fails the
    test instead of skipping it: configs[3] is measured on this file."""
    got, p = S.find_chain(n)
    assert got == n
    return p


def test_sharded_1m_chain_equals_one_batch():
    """BASELINE configs[3] on one GPU: the 1M-round linked chain with 1% of the signatures replaced at
    deterministic positions (a valid signature of another round), verified as one batch and as 8
    contiguous shards (each shard's first link uses sigma_{a-1}, duplicated input, no exchange): the
    concatenated shard bitmaps equal the one-batch bitmap, which flags exactly the corrupted rounds."""
    import torch

    from drand_amd import shard

    N = 1000000
    chain_sigs = np.fromfile(_chain_file(N), dtype=np.uint8).reshape(N, 96)
    bad_pos = np.unique((np.arange(N // 100, dtype=np.int64) * 7919 + 13) % N)
    sigs = chain_sigs.copy()
    sigs[bad_pos] = chain_sigs[(bad_pos + 1) % N]
    rounds = np.arange(1, N + 1, dtype=np.uint64)
    dev = torch.device("cuda", 0)
    lib = L.lib(0)
    pk = S.GROUP_PK
    # prev_sig of round r is the chain's (valid) signature of round r-1: offsets into one buffer
    prev = np.concatenate([np.frombuffer(S.GENESIS_SEED, np.uint8), chain_sigs[:-1].reshape(-1)])
    off = np.concatenate([[0], 32 + 96 * np.arange(N, dtype=np.int64)]).astype(np.int32)
    d_pr = torch.from_numpy((rounds - 1).astype(np.int64)).to(dev)
    d_r = torch.from_numpy(rounds.astype(np.int64)).to(dev)
    d_ps = torch.from_numpy(prev).to(dev)
    d_off = torch.from_numpy(off).to(dev)
    d_sig = torch.from_numpy(sigs).to(dev)
    import ctypes

    def run(lo, hi, seed):
        st = torch.full((hi - lo,), 99, dtype=torch.uint8, device=dev)
        L.check(lib.dg_verify_beacons_dev(ctypes.c_char_p(pk), hi - lo, L.ptr(d_pr[lo:]), L.ptr(d_r[lo:]),
                                          L.ptr(d_ps), L.ptr(d_off[lo:]), L.ptr(d_sig[lo:]), L.ptr(st), seed, None))
        torch.cuda.synchronize()
        return st.cpu().numpy()

    one = run(0, N, 41)
    assert np.nonzero(one)[0].tolist() == bad_pos.tolist()
    assert set(one[bad_pos].tolist()) == {L.ST_BAD_SIG}
    parts = [run(*shard.round_range(N, 8, q), 50 + q) for q in range(8)]
    assert np.array_equal(np.concatenate(parts), one)
    bits = [shard.pack_bits(torch.from_numpy(p)).numpy() for p in parts]
    sizes = [b - a for a, b in (shard.round_range(N, 8, q) for q in range(8))]
    m = max(len(b) for b in bits)
    flat = shard.unpack_bits(np.concatenate([np.pad(b, (0, m - len(b))) for b in bits]), sizes)
    assert np.array_equal(flat, (one != 0).astype(np.uint8))


def test_group_tests_reject_cancelling_errors():
    """Recover's per-item pass checks up to four fresh shares of a round together (random 64-bit weights
    from the bound seed, kernels.h verify_group).  Shares crafted so their errors cancel in the unweighted sum
    (sigma'_0 = sigma_0 + E, sigma'_1 = sigma_1 - E in the same group; E, -2E, +E spread over a group of
    three) fail the weighted group test and are rejected one by one; clean groups pass.  Statuses and
    recovered signatures equal the twin's."""
    t, n, R = 5, 12, 6
    coeffs, commits, shares = group(t, n)
    msgs = [hashlib.sha256(b"grp/%d" % r).digest() for r in range(R)]
    parts = tbls.sign_batch([v for _ in range(R) for _, v in shares], [m for m in msgs for _ in range(n)],
                            [i for _ in range(R) for i, _ in shares]).reshape(R, n, 98)
    E = B.G2C.mul(B.G2_GEN, 24681357)

    def shift(r, j, mult):
        s = B.g2_decompress(bytes(parts[r, j, 2:]))
        parts[r, j, 2:] = np.frombuffer(B.g2_compress(B.G2C.add(s, B.G2C.mul(E, mult % B.R))), np.uint8)

    shift(0, 0, 1), shift(0, 1, -1)                  # one cancelling pair in the first group
    shift(2, 4, 1), shift(2, 5, -2), shift(2, 6, 1)  # three in the second group, sum zero
    shift(3, 1, 3), shift(3, 2, -3), shift(3, 9, 1)  # a pair plus a lone bad share further on
    pub = tbls.PubPoly(commits)
    sigs, rs, ss = tbls.recover_batch(pub, msgs, parts, t, n, seed=21)
    tw = twin.recover_batch(commits, t, n, np.array([list(m) for m in msgs], np.uint8), parts, 8)
    assert np.array_equal(rs, tw[1]) and np.array_equal(ss, tw[2]) and np.array_equal(sigs, tw[0])
    assert ss[0, :2].tolist() == [1, 1] and ss[2, 4:7].tolist() == [1, 1, 1] and ss[3, 1:3].tolist() == [1, 1]
    assert not rs.any() and all(bytes(sigs[r]) == twin.sign(coeffs[0], msgs[r]) for r in range(R))


def test_clean_groups_pass_on_the_group_path():
    """A Recover batch whose batch equation fails for one bad share in round 0: every other round's group
    tests must pass (only round 0's failed group goes to single checks).  Counted with dg_group_counts: a
    failed clean group would add four single checks; at most one tail share per round (t = 5 plus the
    speculative margin) and round 0's rechecks and replacement are checked alone."""
    t, n, R = 5, 12, 40
    coeffs, commits, shares = group(t, n)
    msgs = [hashlib.sha256(b"clean/%d" % r).digest() for r in range(R)]
    parts = tbls.sign_batch([v for _ in range(R) for _, v in shares], [m for m in msgs for _ in range(n)],
                            [i for _ in range(R) for i, _ in shares]).reshape(R, n, 98)
    parts[0, 2, 2:] = np.frombuffer(twin.sign((shares[2][1] + 1) % S.R, msgs[0]), np.uint8)
    pub = tbls.PubPoly(commits)
    g0 = L.group_counts()
    sigs, rs, ss = tbls.recover_batch(pub, msgs, parts, t, n, seed=23)
    g1 = L.group_counts()
    d = [b - a for a, b in zip(g0, g1)]
    assert not rs.any() and ss[0, :6].tolist() == [0, 0, 1, 0, 0, 0]
    if d[3]:  # group tests enabled (DG_GROUP unset)
        assert d[3] >= R and d[0] <= R + 5, d


def test_recover_dev_equals_host_and_twin():
    """dg_recover_dev (messages, partials and outputs in HBM) gives dg_recover's and the twin's signatures,
    round statuses and share statuses, including an index that occurs in fewer than 1/8 of the rounds (checked
    alone) and a duplicated index."""
    import torch

    t, n, R = 5, 12, 24
    coeffs, commits, msgs, parts = _group_rounds(t, n, R, 0.15, b"dev")
    parts[3, 7, :2] = [0, 200]      # a rare index (key slot of its own, outside the batch equation)
    parts[5, 1] = parts[5, 0]      # duplicate index among the first t
    pub = tbls.PubPoly(commits)
    a = tbls.recover_batch(pub, msgs, parts, t, n, seed=41)
    dev = torch.device("cuda", 0)
    d_m = torch.from_numpy(np.array([list(m) for m in msgs], np.uint8)).to(dev)
    d_p = torch.from_numpy(np.ascontiguousarray(parts)).to(dev)
    b = [x.cpu().numpy() for x in tbls.recover_batch_dev(pub, d_m, d_p, t, n, seed=41)]
    for x, y in zip(a, b):
        assert np.array_equal(x, y)
    tw = twin.recover_batch(commits, t, n, np.array([list(m) for m in msgs], np.uint8), parts, 8)
    assert np.array_equal(b[1], tw[1]) and np.array_equal(b[2], tw[2])
    assert np.array_equal(b[0][b[1] == 0], tw[0][tw[1] == 0])


_AB_CHILD = r"""
import json, sys
import numpy as np
sys.path.insert(0, sys.argv[1])
from drand_amd import tbls
from tests.fixtures import chain, chain_arrays, hx
c = chain()
_, _, _, sigs, msgs = chain_arrays(c)
s = sigs[:48].copy()
s[3] = s[4]                      # a valid signature of another round
s[10, 40] ^= 1                   # a flipped bit
s[20] = s[21]
print(json.dumps(tbls.verify_recovered_batch(hx(c["pk"]), msgs[:48], s, seed=5).tolist()))
"""


def test_ab_switches_give_the_same_verdicts():
    """The library's remaining run-time switches reshape the same computation: in a child process with one
    workspace set (DG_SETS=1) and level-1 isolation groups of 2 quads (DG_XR_QPG=2), the verdicts of a corrupted
    batch equal the default library's and the CPU twin's.  (The round-2/3 A/B switches DG_MSM_JAC,
    DG_BINV_CHUNKED, DG_SUB_SEPARATE were removed with their code paths in round 5.)"""
    import json
    import subprocess
    import sys

    c = chain()
    _, _, _, sigs, msgs = chain_arrays(c)
    pk = hx(c["pk"])
    s = sigs[:48].copy()
    s[3] = s[4]
    s[10, 40] ^= 1
    s[20] = s[21]
    here = tbls.verify_recovered_batch(pk, msgs[:48], s, seed=5).tolist()
    want = [twin.verify(pk, bytes(msgs[i]), bytes(s[i])) for i in range(48)]
    assert here == want and sum(1 for v in want if v) == 3
    env = dict(os.environ, DG_SETS="1", DG_XR_QPG="2")
    r = subprocess.run([sys.executable, "-c", _AB_CHILD, ROOT], env=env, capture_output=True, text=True, timeout=240,
                       cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    assert json.loads(r.stdout.strip().splitlines()[-1]) == want


def test_repeated_items_pass_on_the_batch_path():
    """A valid batch whose items repeat (one (message, signature) pair 200 times, then two pairs alternating):
    every MSM bucket holds copies of one point, so the affine levels take the tangent case (P + P) throughout
    and the hash side the same.  The batch equation must hold (no per-item fallback) and every verdict is OK;
    the exact chord / tangent / P + (-P) formulas are also checked on the host
    (test_host_arith.py::test_affine_pair_addition_matches_jacobian)."""
    c = chain()
    _, _, _, sigs, msgs = chain_arrays(c)
    pk = hx(c["pk"])
    for idx in ([0] * 200, [0, 1] * 100):
        m = np.ascontiguousarray(msgs[idx])
        s = np.ascontiguousarray(sigs[idx])
        f0 = L.fallback_count()
        st = tbls.verify_recovered_batch(pk, m, s, seed=9)
        assert not st.any()
        assert L.fallback_count() == f0, "a valid batch of repeated items fell back to the per-item pass"
