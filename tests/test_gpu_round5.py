"""Round-5 parity tests of the HIP path through the C-ABI: the isolation of failed single-key batches by group tests
across rounds (drand_amd/csrc/xr.h) and of failed VerifyPartial batches by the group-test passes of checks.h, against
the CPU twin's per-item bls.Verify / VerifyPartial (kyber decides every beacon and every partial alone:
beacon/chain.go:65-71, beacon/beacon.go:148,575).  Bit-exact statuses.

- the 100k-round linked chain with 1% of the signatures replaced (the c2_negative bench line's positions), verified
  as one batch: exactly the replaced rounds rejected (bad signature), the twin agreeing on them and on a sample;
- every corruption kind in one batch, each in a group test with valid rounds: a signature of another round, of
  another key, undecodable bytes, a flipped x bit (off the curve, or on it outside G2: the failed windowed subgroup
  check sends every signature to k_xg_sub), the identity, a signature repeated for two rounds, a negated signature,
  and an error pair E, -E on neighbouring rounds (they would cancel in an unweighted sum) -- for several seeds and
  level shapes (DG_XR_QPG = 1, 2, 4, 16 in child processes);
- heavy corruption (50%, 100% bad: every round down to its single check, the worst-case capacity of each level);
- a batch across the isolation's segment boundary (140k rounds), growing overlapped batches that regrow workspace
  slots while other batches are in flight, and the workspace of a passing 100k-round batch (round 6);
- asynchronous failed batches overlapped on several workspace sets;
- VerifyPartial with isolated items (a duplicated index in a round, a rare index) and a failed batch, vs the twin."""
import hashlib
import os
import subprocess
import sys

import numpy as np
import pytest

from drand_amd import _lib as L
from drand_amd import tbls
from oracle import twin
from tests.fixtures import chain, chain_arrays, group, hx
from tools import corrupt as C
from tools import synthetic as S

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TW = 16  # twin threads


@pytest.fixture(scope="module", autouse=True)
def device():
    L.lib(0)
    yield


def _signed(R, tag, x=None):
    x = S.master_secret() if x is None else x
    msgs = np.frombuffer(b"".join(hashlib.sha256(b"%s/%d" % (tag, r)).digest() for r in range(R)),
                         np.uint8).reshape(R, 32)
    return x, twin.g1_mul_gen(x), msgs, tbls.sign_batch([x] * R, msgs)


def _mixed(R, tag, touched=None):
    """R GPU-signed rounds of one key with every corruption kind at known positions (the rest valid); `touched`, when
    given, receives every position the corruption wrote."""
    from oracle.pyref import bls12381 as B

    x, pk, msgs, sigs = _signed(R, tag)
    bad = sigs.copy()
    rng = np.random.default_rng(int.from_bytes(hashlib.sha256(tag).digest()[:4], "big"))
    pos = rng.choice(R, size=R // 16, replace=False)
    kinds = []
    other = tbls.sign_batch([x + 1] * len(pos), msgs[pos])  # another key's signatures
    touched = set() if touched is None else touched
    for q, p in enumerate(pos.tolist()):
        kind = q % 8
        touched.update({p, (p + 7) % R} if kind == 5 else {p, (p + 1) % R} if kind == 7 else {p})
        if kind == 0:
            bad[p] = sigs[(p + 1) % R]                                    # another round's signature
        elif kind == 1:
            bad[p] = other[q]                                             # another key's
        elif kind == 2:
            bad[p] = np.frombuffer(hashlib.sha256(b"rb%d" % p).digest() * 3, np.uint8)  # random bytes
        elif kind == 3:
            bad[p, 40] ^= 0x04                                           # a flipped x bit
        elif kind == 4:
            bad[p] = 0
            bad[p, 0] = 0xC0                                              # the identity
        elif kind == 5:
            bad[p] = sigs[(p + 7) % R]                                    # repeated for another round too
            bad[(p + 7) % R] = sigs[(p + 7) % R]
        elif kind == 6:
            bad[p] = sigs[p]
            bad[p, 0] ^= 0x20                                             # negated
        else:
            # an error pair on neighbouring rounds: sigma_p + E and sigma_{p+1} - E (E = round 0's signature, in G2)
            e = B.g2_decompress(bytes(sigs[0]), subgroup_check=False)
            a = B.G2C.add(B.g2_decompress(bytes(sigs[p]), subgroup_check=False), e)
            b = B.G2C.add(B.g2_decompress(bytes(sigs[(p + 1) % R]), subgroup_check=False), B.G2C.neg(e))
            bad[p] = np.frombuffer(B.g2_compress(a), np.uint8)
            bad[(p + 1) % R] = np.frombuffer(B.g2_compress(b), np.uint8)
        kinds.append(kind)
    want = twin.verify_batch(pk, msgs, bad, threads=TW)
    return pk, msgs, bad, want


def test_chain_100k_one_percent_replaced_vs_twin():
    """configs[1] negative: the 100k-round linked chain with 1% of the signatures replaced by the
    next round's (the positions of bench.py's c2_negative line) as one dg_verify_beacons_dev batch: exactly those
    rounds rejected as bad signatures, the rest valid; the twin agrees on every replaced round and on 4000 others;
    the isolation ran its levels (dg_isolation_counts) far below one check per round."""
    import torch

    N = 100000
    n_, path_ = S.find_chain(N)
    sigs = np.fromfile(path_, dtype=np.uint8).reshape(n_, 96)[:N]
    bad_pos = np.unique((np.arange(N // 100, dtype=np.int64) * 7919 + 13) % N)
    bad = sigs.copy()
    bad[bad_pos] = sigs[np.where(bad_pos + 1 < N, bad_pos + 1, bad_pos - 1)]
    rounds = np.arange(1, N + 1, dtype=np.uint64)
    prev = np.concatenate([np.frombuffer(S.GENESIS_SEED, np.uint8), sigs[:-1].reshape(-1)])
    off = np.concatenate([[0], 32 + 96 * np.arange(N, dtype=np.int64)]).astype(np.int32)
    dev = torch.device("cuda", 0)
    d = [torch.from_numpy(a).to(dev) for a in ((rounds - 1).astype(np.int64), rounds.astype(np.int64), prev, off, bad)]
    st = torch.full((N,), 99, dtype=torch.uint8, device=dev)
    lib = L.lib(0)
    x0 = L.isolation_counts()
    L.check(lib.dg_verify_beacons_dev(S.GROUP_PK, N, L.ptr(d[0]), L.ptr(d[1]), L.ptr(d[2]), L.ptr(d[3]), L.ptr(d[4]),
                                      L.ptr(st), 77, None))
    torch.cuda.synchronize()
    x1 = L.isolation_counts()
    got = st.cpu().numpy()
    assert np.nonzero(got)[0].tolist() == bad_pos.tolist()
    assert set(got[bad_pos].tolist()) == {L.ST_BAD_SIG}
    checks = [b - a for a, b in zip(x0, x1)]
    assert checks[2] >= len(bad_pos) and sum(checks) < N // 4, checks
    # the twin on the replaced rounds and a sample of the others
    msgs = tbls.beacon_messages(rounds - 1, rounds, [S.GENESIS_SEED] + [bytes(s) for s in sigs[:-1]])
    rng = np.random.default_rng(5)
    sample = np.unique(np.concatenate([bad_pos, rng.choice(N, 4000, replace=False)]))
    tw = twin.verify_batch(S.GROUP_PK, msgs[sample], bad[sample], threads=TW)
    assert np.array_equal(got[sample], tw)


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_mixed_corruption_in_group_tests_vs_twin(seed):
    """Every corruption kind, ~1/16 of 4096 rounds (so most group tests of 16 and 4 rounds hold a bad round beside
    valid ones), one batch: statuses equal the twin's per-item bls.Verify, for three seeds.  The valid rounds come from
    the GPU's dg_sign, so the twin's verdict on every untouched round is asserted valid first: a wrong dg_sign cannot
    pass with a verifier that agrees with it."""
    touched = set()
    pk, msgs, bad, want = _mixed(4096, b"mix%d" % seed, touched)
    untouched = np.setdiff1d(np.arange(4096), np.array(sorted(touched)))
    assert len(untouched) > 3500 and (want[untouched] == 0).all()
    assert (want == L.ST_BAD_SIG).sum() > 100 and (want == L.ST_SIG_DECODE).sum() > 50
    st = tbls.verify_recovered_batch(pk, msgs, bad, seed=seed)
    assert np.array_equal(st, want)
    assert L.last_batch_flags()[0] is False


def test_failed_batch_after_passed_batches_narrow_grids():
    """A failed batch right after passed ones on the same context (blocking calls: each batch's isolation workspace
    reused by the next), ~2 k single checks at level 3: the statuses equal the twin's; then the same batch again."""
    pk, msgs, bad, want = _mixed(4096, b"narrow")
    x, pk2, msgs2, sigs2 = _signed(512, b"narrow-clean")
    for _ in range(2):
        assert not tbls.verify_recovered_batch(pk2, msgs2, sigs2, seed=5).any()
    x0 = L.isolation_counts()
    st = tbls.verify_recovered_batch(pk, msgs, bad, seed=6)
    x1 = L.isolation_counts()
    assert np.array_equal(st, want)
    assert x1[2] - x0[2] > 1024, (x0, x1)
    assert np.array_equal(tbls.verify_recovered_batch(pk, msgs, bad, seed=7), want)


_QPG_CHILD = r"""
import sys
import numpy as np
sys.path.insert(0, sys.argv[1])
from drand_amd import _lib as L
from drand_amd import tbls
z = np.load(sys.argv[2])
L.lib(0)
st = tbls.verify_recovered_batch(bytes(z["pk"]), z["msgs"], z["sigs"], seed=int(z["seed"]))
np.save(sys.argv[3], st)
"""


@pytest.mark.parametrize("shape", [{"DG_XR_QPG": "1"}, {"DG_XR_QPG": "2"}, {"DG_XR_QPG": "16"}],
                         ids=["quads", "qpg2", "qpg16"])
def test_level_shapes_vs_twin(tmp_path, shape):
    """The isolation's level shapes in a child process (DG_XR_QPG: level-1 groups of 1, 2 or 16 quads, i.e. 4, 8 or 64
    rounds, then every round of a failed group alone): the same statuses as the twin on a mixed batch."""
    pk, msgs, bad, want = _mixed(2048, b"qpg" + "".join(shape.values()).encode())
    inp, out = tmp_path / "in.npz", tmp_path / "out.npy"
    np.savez(inp, pk=np.frombuffer(pk, np.uint8), msgs=msgs, sigs=bad, seed=9)
    r = subprocess.run([sys.executable, "-c", _QPG_CHILD, ROOT, str(inp), str(out)],
                       env=dict(os.environ, **shape), capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    assert np.array_equal(np.load(out), want)


@pytest.mark.parametrize("frac", [0.5, 1.0])
def test_heavy_corruption_every_level_at_capacity(frac):
    """Half, then all of 2048 rounds carry another round's signature: every group test and quad fails, so the single
    checks of the last level hold up to every round of the batch (the capacity each level is launched with)."""
    R = 2048
    x, pk, msgs, sigs = _signed(R, b"heavy")
    n = int(R * frac)
    pos = np.sort(np.random.default_rng(3).choice(R, n, replace=False))
    bad = sigs.copy()
    bad[pos] = sigs[(pos + 1) % R]
    want = np.zeros(R, np.uint8)
    want[pos] = L.ST_BAD_SIG
    x0 = L.isolation_counts()
    st = tbls.verify_recovered_batch(pk, msgs, bad, seed=11)
    x1 = L.isolation_counts()
    assert np.array_equal(st, want)
    assert x1[2] - x0[2] >= n
    tw = twin.verify_batch(pk, msgs[:256], bad[:256], threads=TW)
    assert np.array_equal(st[:256], tw)


def test_isolation_segment_boundary_140k():
    """Round-5 advice: a batch longer than one isolation segment (kXrSeg = 131072 items): 140k rounds of the linked
    chain with replaced signatures on both sides of item 131072 (131071, 131072, 131073, and a few in each segment):
    exactly those rounds rejected, the twin agreeing on them and on their neighbours."""
    import torch

    N = 140000
    n_, path_ = S.find_chain(N)
    sigs = np.fromfile(path_, dtype=np.uint8).reshape(n_, 96)[:N]
    bad_pos = np.array(sorted({5, 70000, 131070, 131071, 131072, 131073, 135000, N - 1}))
    bad = sigs.copy()
    bad[bad_pos] = sigs[np.where(bad_pos + 1 < N, bad_pos + 1, bad_pos - 1)]
    rounds = np.arange(1, N + 1, dtype=np.uint64)
    prev = np.concatenate([np.frombuffer(S.GENESIS_SEED, np.uint8), sigs[:-1].reshape(-1)])
    off = np.concatenate([[0], 32 + 96 * np.arange(N, dtype=np.int64)]).astype(np.int32)
    dev = torch.device("cuda", 0)
    d = [torch.from_numpy(a).to(dev) for a in ((rounds - 1).astype(np.int64), rounds.astype(np.int64), prev, off, bad)]
    st = torch.full((N,), 99, dtype=torch.uint8, device=dev)
    lib = L.lib(0)
    L.check(lib.dg_verify_beacons_dev(S.GROUP_PK, N, L.ptr(d[0]), L.ptr(d[1]), L.ptr(d[2]), L.ptr(d[3]), L.ptr(d[4]),
                                      L.ptr(st), 91, None))
    torch.cuda.synchronize()
    got = st.cpu().numpy()
    assert np.nonzero(got)[0].tolist() == bad_pos.tolist()
    assert set(got[bad_pos].tolist()) == {L.ST_BAD_SIG}
    sample = np.unique(np.clip(np.concatenate([bad_pos - 1, bad_pos, bad_pos + 1]), 0, N - 1))
    msgs = tbls.beacon_messages(rounds[sample] - 1, rounds[sample], [S.GENESIS_SEED if i == 0 else bytes(sigs[i - 1])
                                                                    for i in sample])
    tw = twin.verify_batch(S.GROUP_PK, msgs, bad[sample], threads=TW)
    assert np.array_equal(got[sample], tw)


def test_overlapped_failed_batches_with_slot_regrowth():
    """Round-5 verdict item 4: asynchronous batches of GROWING size (1000 .. 12000 rounds of the linked chain, every
    other one with replaced signatures) rotating over the workspace sets, drained once.  Each set and each tail
    stream's isolation workspace regrows while batches of other sets -- and, on the shared tail streams, their
    isolations -- are still in flight; every status buffer flags exactly its replaced rounds."""
    import torch

    n_, path_ = S.find_chain(12000)
    chain_sigs = np.fromfile(path_, dtype=np.uint8).reshape(n_, 96)[:12000]
    N = 12000
    rounds = np.arange(1, N + 1, dtype=np.uint64)
    prev = np.concatenate([np.frombuffer(S.GENESIS_SEED, np.uint8), chain_sigs[:-1].reshape(-1)])
    off = np.concatenate([[0], 32 + 96 * np.arange(N, dtype=np.int64)]).astype(np.int32)
    dev = torch.device("cuda", 0)
    d_pr = torch.from_numpy((rounds - 1).astype(np.int64)).to(dev)
    d_r = torch.from_numpy(rounds.astype(np.int64)).to(dev)
    d_ps = torch.from_numpy(prev).to(dev)
    d_off = torch.from_numpy(off).to(dev)
    lib = L.lib(0)
    outs = []
    for k in range(12):
        n = 1000 * (k + 1)
        sigs = chain_sigs[:n].copy()
        pos = np.array([], np.int64)
        if k % 2:
            pos = np.unique((np.arange(k + 3) * 977 + 31 * k) % n)
            sigs[pos] = chain_sigs[(pos + 1) % n]
        d_sig = torch.from_numpy(sigs).to(dev)
        d_st = torch.full((n,), 99, dtype=torch.uint8, device=dev)
        torch.cuda.synchronize()
        L.check(lib.dg_verify_beacons_dev_async(S.GROUP_PK, n, L.ptr(d_pr), L.ptr(d_r), L.ptr(d_ps), L.ptr(d_off),
                                                L.ptr(d_sig), L.ptr(d_st), 300 + k, None, None))
        outs.append((n, pos, d_sig, d_st))
    L.check(lib.dg_wait_all())
    torch.cuda.synchronize()
    for k, (n, pos, _, d_st) in enumerate(outs):
        got = d_st.cpu().numpy()
        assert np.nonzero(got)[0].tolist() == pos.tolist(), k
        assert set(got[pos].tolist()) <= {L.ST_BAD_SIG}, k


_PASSING_MEM_CHILD = r"""
import sys
import numpy as np
sys.path.insert(0, sys.argv[1])
import torch
from drand_amd import _lib as L
from tools import synthetic as S
lib = L.lib(0)
N = 100000
n_, path_ = S.find_chain(N)
sigs = np.fromfile(path_, dtype=np.uint8).reshape(n_, 96)[:N]
rounds = np.arange(1, N + 1, dtype=np.uint64)
prev = np.concatenate([np.frombuffer(S.GENESIS_SEED, np.uint8), sigs[:-1].reshape(-1)])
off = np.concatenate([[0], 32 + 96 * np.arange(N, dtype=np.int64)]).astype(np.int32)
dev = torch.device("cuda", 0)
d = [torch.from_numpy(a).to(dev) for a in ((rounds - 1).astype(np.int64), rounds.astype(np.int64), prev, off, sigs)]
st = torch.full((N,), 99, dtype=torch.uint8, device=dev)
torch.cuda.synchronize()
free0 = torch.cuda.mem_get_info(0)[0]
L.check(lib.dg_verify_beacons_dev_async(S.GROUP_PK, N, L.ptr(d[0]), L.ptr(d[1]), L.ptr(d[2]), L.ptr(d[3]),
                                        L.ptr(d[4]), L.ptr(st), 5, None, None))
L.check(lib.dg_wait_all())
torch.cuda.synchronize()
free1 = torch.cuda.mem_get_info(0)[0]
assert not st.cpu().numpy().any()
print(free0 - free1)
"""


def test_passing_100k_batch_workspace_bounded():
    """Round-5 advice (medium): a PASSING 100k-round asynchronous batch on a fresh context takes the workspace of one
    set plus its tail stream's isolation workspace -- sized for the worst case, every round a single check, but ~5 KB a
    check now that no line table is stored (xr.h k_xg_miller): under 3.5 GB (round 5: ~45 KB a check, the isolation
    alone ~4.5 GB of every workspace set at 100k rounds)."""
    r = subprocess.run([sys.executable, "-c", _PASSING_MEM_CHILD, ROOT], capture_output=True, text=True, timeout=300,
                       cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    used = int(r.stdout.strip().splitlines()[-1])
    print("workspace of one passing 100k-round batch: %.2f GB" % (used / 1e9))
    assert used < int(3.5 * (1 << 30)), used


def test_async_failed_batches_overlapped():
    """Six asynchronous batches of the committed chain on rotating workspace sets, every other one with corrupted
    rounds (its isolation enqueued whole on the batch's stream, no host round trip), drained once: each status buffer
    equals the twin's verdicts."""
    import torch

    c = chain()
    pr, rr, ps, sigs, msgs = chain_arrays(c)
    pk = hx(c["pk"])
    bad = sigs.copy()
    bad[3] = sigs[4]
    bad[17, 40] ^= 0x04
    bad[40] = sigs[40]
    bad[40, 0] ^= 0x20
    want_bad = np.array([twin.verify(pk, bytes(msgs[i]), bytes(bad[i])) for i in range(len(rr))], np.uint8)
    dev = torch.device("cuda", 0)
    p_, r_, psb, off = tbls._beacon_arrays(pr, rr, ps)
    d_pr = torch.from_numpy(p_.astype(np.int64)).to(dev)
    d_r = torch.from_numpy(r_.astype(np.int64)).to(dev)
    d_ps = torch.from_numpy(psb).to(dev)
    d_off = torch.from_numpy(off.astype(np.int32)).to(dev)
    n = len(rr)
    lib = L.lib()
    outs = []
    for k in range(6):
        d_sig = torch.from_numpy(np.ascontiguousarray(bad if k % 2 else sigs)).to(dev)
        d_st = torch.full((n,), 99, dtype=torch.uint8, device=dev)
        torch.cuda.synchronize()
        L.check(lib.dg_verify_beacons_dev_async(L.ptr(pk), n, L.ptr(d_pr), L.ptr(d_r), L.ptr(d_ps), L.ptr(d_off),
                                                L.ptr(d_sig), L.ptr(d_st), 60 + k, None, None))
        outs.append((k, d_sig, d_st))
    L.check(lib.dg_wait_all())
    torch.cuda.synchronize()
    for k, _, d_st in outs:
        exp = want_bad if k % 2 else np.zeros(n, np.uint8)
        assert np.array_equal(d_st.cpu().numpy(), exp), k


def test_verify_partials_isolated_and_failed_vs_twin():
    """VerifyPartial (n = 24, t = 9, 32 rounds): a passed batch with isolated items (a second partial with an index
    already used in its round; an index seen in one round only, checked alone), then the same partials with 15%
    corrupted (a failed batch: every partial through the group-test passes): every status equals the twin's."""
    t, n, R = 9, 24, 32
    coeffs, commits, shares = group(t, n)
    msgs = [hashlib.sha256(b"vpi/%d" % r).digest() for r in range(R)]
    parts = tbls.sign_batch([v for _ in range(R) for _, v in shares], [m for m in msgs for _ in range(n)],
                            [i for _ in range(R) for i, _ in shares]).reshape(R, n, 98)
    parts[5, 3] = parts[5, 2]                       # a duplicated (index, sigma) in round 5
    rare = tbls.sign_batch([S.share_value(coeffs, 200)], [msgs[9]], [200])
    parts[9, 7] = rare[0]                           # index 200, seen in this round only
    pub = tbls.PubPoly(commits)
    want = np.array([[twin.verify_partial(commits, msgs[r], bytes(parts[r, j])) for j in range(n)] for r in range(R)])
    st = tbls.verify_partial_batch(pub, msgs, parts, seed=3)
    assert np.array_equal(st, want) and want[9, 7] == 0
    assert L.last_batch_flags() == (True, True)     # passed, with isolated items

    def resign(reqs):
        return tbls.sign_batch([(shares[i][1] + ds) % S.R for (r, i, ds, dr) in reqs],
                               [msgs[(r + dr) % R] if dr else msgs[r] for (r, i, ds, dr) in reqs])

    C.corrupt_batch(parts, C.pick(R, n, 0.15, seed=b"vpi"), n, resign)
    want = np.array([[twin.verify_partial(commits, msgs[r], bytes(parts[r, j])) for j in range(n)] for r in range(R)])
    for seed in (4, 5):
        st = tbls.verify_partial_batch(pub, msgs, parts, seed=seed)
        assert np.array_equal(st, want), seed
    assert (want == L.ST_BAD_SIG).sum() > 10


def test_reference_test_json_points_through_the_kernels():
    """The reference's test/test-integration/test.json points through the device decoders (tests/golden/
    reference_test_json_points.json): its two G1 signatures as the group key of dg_verify (k_decode_g1) and its G2
    `Public` as the signature (the sigma decode phases) give a pairing failure, status 1 -- both decode; Public with its
    c0 / c1 halves swapped, its compression flag cleared or its infinity flag set is a decode error (2); with its sign
    flag flipped, a valid point again (1).  Each equal to the twin's bls.Verify."""
    from tests.test_oracle import _g2_variants, _ref_points

    pub, prev, sig = _ref_points()
    msgs = np.frombuffer(hashlib.sha256(b"test.json").digest() * 8, np.uint8).reshape(8, 32)
    vs = _g2_variants(pub)
    sigs = np.frombuffer(pub + b"".join(vs.values()) + pub * 3, np.uint8).reshape(8, 96)
    for key in (prev, sig):
        want = twin.verify_batch(key, msgs, sigs, threads=4)
        assert want.tolist() == [1, 2, 2, 2, 1, 1, 1, 1]
        for seed in (1, 2):
            assert tbls.verify_recovered_batch(key, msgs, sigs, seed=seed).tolist() == want.tolist()


_SMALL_RECOVER_CHILD = r"""
import hashlib, sys
import numpy as np
sys.path.insert(0, sys.argv[1])
import torch
from drand_amd import _lib as L
from drand_amd import tbls
from tests.fixtures import group
L.lib(0)
torch.cuda.synchronize()
free0 = torch.cuda.mem_get_info(0)[0]
t, n, R = 3, 5, 4
coeffs, commits, shares = group(t, n)
msgs = [hashlib.sha256(b"small/%d" % r).digest() for r in range(R)]
parts = tbls.sign_batch([v for _ in range(R) for _, v in shares], [m for m in msgs for _ in range(n)],
                        [i for _ in range(R) for i, _ in shares]).reshape(R, n, 98)
parts[1, 0] = parts[2, 0]  # one share carries another round's partial
sigs, rs, ss = tbls.recover_batch(tbls.PubPoly(commits), msgs, parts, t, n, seed=5)
torch.cuda.synchronize()
free1 = torch.cuda.mem_get_info(0)[0]
assert not rs.any() and ss[1, 0] != 0 and (ss[0, :t] == 0).all(), (rs, ss)
print(free0 - free1)
"""


def test_small_recover_keeps_workspace_small(tmp_path):
    """Round-4 advice (medium): a small Recover with one corrupted share (its per-item pass runs) sizes the check
    pipeline's buffers for the checks it runs, not for CK_CHUNK: the device memory it takes on a fresh set 0 stays far
    below 1 GB (a fresh process, torch.cuda.mem_get_info around the first call)."""
    r = subprocess.run([sys.executable, "-c", _SMALL_RECOVER_CHILD, ROOT], capture_output=True, text=True, timeout=300,
                       cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    used = int(r.stdout.strip().splitlines()[-1])
    assert used < (1 << 30), used
