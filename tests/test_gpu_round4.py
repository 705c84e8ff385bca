"""Round-4 parity tests of the HIP path through the C-ABI, against the CPU twin's tbls.Recover (signatures, round
statuses, every share status; bit-exact):

- Recover at C3's exact shape (BASELINE configs[2]: n = 64, t = 33, partials in index order): every 64-round block
  selects the consecutive index set 0..32, so recover.h's uniform Straus path runs with the negated-binomial
  Lagrange coefficients (the ~31-bit d0 case) -- before this round it was twin-checked only at t <= 8;
- a batch whose uniform and divergent 64-round blocks coexist (R % 64 != 0, one corrupted window share in a middle
  block, a NOT_ENOUGH round inside an otherwise uniform block: the ub / nl block lists of recover_tail);
- the exact per-item mode (DG_GROUP=1: every examined share gets its own pairing check, no group tests) at a C5
  shape (n = 256, t = 129, 30% corrupted) in a child process;
- the HBM-resident VerifyPartial + Recover-from-verdicts pair that bench.py times as configs[2];
- the per-item pass in its schedule variants (child processes: no speculative passes, DG_CK_PASSES=0, so every
  unverified share takes the final pass alone; no first-pass margin, DG_CK_MARGIN0=0) with repeated and cancelling
  members inside group tests;
- asynchronous beacon batches consumed on the batch's own stream (dg_last_batch_stream)."""
import hashlib
import json
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


def _in_order(t, n, R, label):
    coeffs, commits, shares = group(t, n)
    msgs = [hashlib.sha256(b"%s/%d" % (label, r)).digest() for r in range(R)]
    parts = tbls.sign_batch([v for _ in range(R) for _, v in shares], [m for m in msgs for _ in range(n)],
                            [i for _ in range(R) for i, _ in shares]).reshape(R, n, 98)
    return coeffs, commits, msgs, parts


def _twin(commits, t, n, msgs, parts):
    return twin.recover_batch(commits, t, n, np.array([list(m) for m in msgs], np.uint8), parts, TW)


def _equal(got, tw):
    sigs, rs, ss = got
    assert np.array_equal(rs, tw[1])
    assert np.array_equal(ss, tw[2])
    assert np.array_equal(sigs[rs == 0], tw[0][tw[1] == 0])


def test_recover_c3_shape_uniform_blocks_vs_twin():
    """n = 64, t = 33, 129 clean rounds in index order: two full uniform blocks and a one-round block, all on the
    consecutive set 0..32 (recover.h: the negated binomial coefficients); the batch equation holds (fast path)."""
    t, n, R = 33, 64, 129
    coeffs, commits, msgs, parts = _in_order(t, n, R, b"c3u")
    f0 = L.fallback_count()
    got = tbls.recover_batch(tbls.PubPoly(commits), msgs, parts, t, n, seed=31)
    assert L.fallback_count() == f0, "a clean C3 batch left the batch path"
    _equal(got, _twin(commits, t, n, msgs, parts))
    assert not got[1].any() and (got[2][:, :t] == 0).all() and (got[2][:, t:] == 255).all()
    for r in (0, 63, 64, 128):
        assert bytes(got[0][r]) == twin.sign(coeffs[0], msgs[r])


def test_recover_uniform_and_divergent_blocks_coexist():
    """200 rounds in index order (R % 64 = 8): round 70 has another round's partial at position 5 of its window
    (block 1 selects a different set there: divergent), round 10 has fewer than t decodable shares (NOT_ENOUGH
    inside the otherwise uniform block 0), round 140 has an undecodable share beyond its window (block 2 stays
    uniform); blocks 0, 2 and the partial block 3 take the uniform path, block 1 the joint column MSM."""
    t, n, R = 33, 64, 200
    coeffs, commits, msgs, parts = _in_order(t, n, R, b"c3mix")
    parts[70, 5] = parts[71, 5]
    parts[10, :n - t + 1, 2:] = 0xff
    parts[140, 50, 2:] = 0xff
    got = tbls.recover_batch(tbls.PubPoly(commits), msgs, parts, t, n, seed=32)
    _equal(got, _twin(commits, t, n, msgs, parts))
    rs, ss = got[1], got[2]
    assert np.nonzero(rs)[0].tolist() == [10] and rs[10] == L.ST_NOT_ENOUGH
    assert ss[70, 5] == L.ST_BAD_SIG and ss[70, t] == 0 and ss[140, 50] == 255
    for r in (0, 63, 70, 127, 199):
        assert bytes(got[0][r]) == twin.sign(coeffs[0], msgs[r])


_EXACT_CHILD = r"""
import json, sys
import numpy as np
sys.path.insert(0, sys.argv[1])
from drand_amd import _lib as L
from drand_amd import tbls
z = np.load(sys.argv[2])
commits = [bytes(c) for c in z["commits"]]
g0 = L.group_counts()
sigs, rs, ss = tbls.recover_batch(tbls.PubPoly(commits), z["msgs"], z["parts"], int(z["t"]), int(z["n"]), seed=33)
g1 = L.group_counts()
np.savez(sys.argv[3], sigs=sigs, rs=rs, ss=ss, counts=np.array([b - a for a, b in zip(g0, g1)]))
"""


def test_exact_group_mode_c5_shape_vs_twin(tmp_path):
    """DG_GROUP=1 (child process): Recover's per-item pass checks every examined share alone -- exact verdicts, no
    group test -- at n = 256, t = 129 with 30% of the shares corrupted by the six modes of tools/corrupt.py; the
    statuses and signatures equal the twin's and the default (group-test) library's."""
    t, n, R = 129, 256, 8
    coeffs, commits, shares = group(t, n)
    msgs = [hashlib.sha256(b"exact/%d" % r).digest() for r in range(R)]
    parts = tbls.sign_batch([v for _ in range(R) for _, v in shares], [m for m in msgs for _ in range(n)],
                            [i for _ in range(R) for i, _ in shares]).reshape(R, n, 98)

    def resign(reqs):
        return tbls.sign_batch([(shares[i][1] + ds) % S.R for (r, i, ds, dr) in reqs],
                               [msgs[(r + dr) % R] if dr else msgs[r] for (r, i, ds, dr) in reqs])

    C.corrupt_batch(parts, C.pick(R, n, 0.30, seed=b"exact"), n, resign)
    inp = tmp_path / "in.npz"
    out = tmp_path / "out.npz"
    np.savez(inp, commits=np.array([list(c) for c in commits], np.uint8), msgs=np.array([list(m) for m in msgs],
             np.uint8), parts=parts, t=t, n=n)
    env = dict(os.environ, DG_GROUP="1")
    r = subprocess.run([sys.executable, "-c", _EXACT_CHILD, ROOT, str(inp), str(out)], env=env, capture_output=True,
                       text=True, timeout=300, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    z = np.load(out)
    tw = _twin(commits, t, n, msgs, parts)
    _equal((z["sigs"], z["rs"], z["ss"]), tw)
    assert z["counts"][0] > 0 and not z["counts"][1:].any(), "DG_GROUP=1 ran group tests"
    dflt = tbls.recover_batch(tbls.PubPoly(commits), msgs, parts, t, n, seed=33)
    _equal(dflt, tw)
    assert (z["ss"] != 255).sum() >= t * R


def test_verify_partials_dev_and_recover_from_verdicts():
    """The configs[2] pair bench.py times: dg_verify_partials_dev over every partial (HBM-resident) equals the
    host-buffer dg_verify_partials and the twin's VerifyPartial, and dg_recover_verified_dev from those verdicts
    equals dg_recover (and so the twin's Recover)."""
    import torch

    t, n, R = 5, 12, 70
    coeffs, commits, shares = group(t, n)
    msgs = [hashlib.sha256(b"vpdev/%d" % r).digest() for r in range(R)]
    parts = tbls.sign_batch([v for _ in range(R) for _, v in shares], [m for m in msgs for _ in range(n)],
                            [i for _ in range(R) for i, _ in shares]).reshape(R, n, 98)

    def resign(reqs):
        return tbls.sign_batch([(shares[i][1] + ds) % S.R for (r, i, ds, dr) in reqs],
                               [msgs[(r + dr) % R] if dr else msgs[r] for (r, i, ds, dr) in reqs])

    C.corrupt_batch(parts, C.pick(R, n, 0.2, seed=b"vpdev"), n, resign)
    pub = tbls.PubPoly(commits)
    host = tbls.verify_partial_batch(pub, msgs, parts, seed=34)
    dev = torch.device("cuda", 0)
    d_m = torch.from_numpy(np.array([list(m) for m in msgs], np.uint8)).to(dev)
    d_p = torch.from_numpy(np.ascontiguousarray(parts)).to(dev)
    d_st = tbls.verify_partial_batch_dev(pub, d_m, d_p, seed=34)
    assert np.array_equal(d_st.cpu().numpy(), host)
    want = np.array([[twin.verify_partial(commits, msgs[r], bytes(parts[r, j])) for j in range(n)] for r in range(R)])
    assert np.array_equal(host, want) and want.any()
    a = tbls.recover_batch(pub, msgs, parts, t, n, seed=34)
    b = [x.cpu().numpy() for x in tbls.recover_verified_batch_dev(d_p, d_st, t, n)]
    for x, y in zip(a, b):
        assert np.array_equal(x, y)
    _equal(b, _twin(commits, t, n, msgs, parts))


def test_wrong_length_placeholder_is_skipped():
    """gpu/scheme.go (VerifyPartialBatch, RecoverBatch) sends a partial of the wrong length as a 98 B placeholder
    (index 0, sigma without the compression flag): the library must report it as a decode error and Recover must
    skip it exactly as kyber's tbls.Recover skips an unparsable partial -- the same signature as with the partial
    left out, and the twin's statuses."""
    t, n, R = 5, 12, 4
    coeffs, commits, msgs, parts = _in_order(t, n, R, b"short")
    ph = np.zeros(98, np.uint8)
    bad = parts.copy()
    bad[1, 2] = ph
    bad[3, 0] = ph
    pub = tbls.PubPoly(commits)
    st = tbls.verify_partial_batch(pub, msgs, bad, seed=35)
    assert st[1, 2] == L.ST_SIG_DECODE and st[3, 0] == L.ST_SIG_DECODE and st.sum() == 2 * L.ST_SIG_DECODE
    sigs, rs, ss = tbls.recover_batch(pub, msgs, bad, t, n, seed=35)
    _equal((sigs, rs, ss), _twin(commits, t, n, msgs, bad))
    assert not rs.any() and ss[1, 2] == L.ST_SIG_DECODE and ss[1, t] == 0
    for r in range(R):
        assert bytes(sigs[r]) == twin.sign(coeffs[0], msgs[r])


_FORM_CHILD = r"""
import sys
import numpy as np
sys.path.insert(0, sys.argv[1])
from drand_amd import _lib as L
from drand_amd import tbls
z = np.load(sys.argv[2])
commits = [bytes(c) for c in z["commits"]]
sigs, rs, ss = tbls.recover_batch(tbls.PubPoly(commits), z["msgs"], z["parts"], int(z["t"]), int(z["n"]), seed=36)
np.savez(sys.argv[3], sigs=sigs, rs=rs, ss=ss)
"""


def test_pipeline_forms_with_repeated_and_cancelling_members(tmp_path):
    """n = 256, t = 129, 8 rounds, 15% corrupted, plus members that repeat (a partial copied whole over its neighbour:
    the same sigma twice in one group test -- the affine table's tangent case) and cancel (a neighbour's sigma
    negated: P + (-P) = O in the table) inside the examined prefix.  The default library and child processes with
    the schedule variants of the per-item pass all give the twin's signatures and statuses."""
    t, n, R = 129, 256, 8
    coeffs, commits, shares = group(t, n)
    msgs = [hashlib.sha256(b"forms/%d" % r).digest() for r in range(R)]
    parts = tbls.sign_batch([v for _ in range(R) for _, v in shares], [m for m in msgs for _ in range(n)],
                            [i for _ in range(R) for i, _ in shares]).reshape(R, n, 98)

    def resign(reqs):
        return tbls.sign_batch([(shares[i][1] + ds) % S.R for (r, i, ds, dr) in reqs],
                               [msgs[(r + dr) % R] if dr else msgs[r] for (r, i, ds, dr) in reqs])

    C.corrupt_batch(parts, C.pick(R, n, 0.15, seed=b"forms"), n, resign)
    for r in range(R):
        j = 8 + 12 * r
        parts[r, j] = parts[r, j + 1]                # the same partial twice (index included)
        parts[r, j + 4] = parts[r, j + 5]
        parts[r, j + 4, 2] ^= 0x20                   # ... and a neighbour's sigma negated (index j + 5)
    tw = _twin(commits, t, n, msgs, parts)
    assert (tw[2] == L.ST_BAD_SIG).any()
    _equal(tbls.recover_batch(tbls.PubPoly(commits), msgs, parts, t, n, seed=36), tw)
    inp = tmp_path / "in.npz"
    np.savez(inp, commits=np.array([list(c) for c in commits], np.uint8), msgs=np.array([list(m) for m in msgs],
             np.uint8), parts=parts, t=t, n=n)
    for k, (var, val) in enumerate([("DG_CK_PASSES", "0"), ("DG_CK_MARGIN0", "0")]):
        out = tmp_path / ("out%d.npz" % k)
        r = subprocess.run([sys.executable, "-c", _FORM_CHILD, ROOT, str(inp), str(out)],
                           env=dict(os.environ, **{var: val}), capture_output=True, text=True, timeout=300, cwd=ROOT)
        assert r.returncode == 0, (var, r.stderr[-2000:])
        z = np.load(out)
        _equal((z["sigs"], z["rs"], z["ss"]), tw)


def test_async_batches_consumed_on_the_batch_stream():
    """dg_verify_beacons_dev_async without a done stream, its statuses packed on dg_last_batch_stream()'s stream
    (bench.py's arrangement at N = 1): four overlapped batches of the committed chain, one of them corrupted, equal
    the blocking entry point's statuses and the twin's."""
    import ctypes

    import torch

    from drand_amd import shard

    c = chain()
    pr, rr, ps, sigs, msgs = chain_arrays(c)
    pk = hx(c["pk"])
    bad = sigs.copy()
    bad[3] = sigs[4]
    bad[7, 0] ^= 0x20
    want = [twin.verify(pk, bytes(msgs[i]), bytes(bad[i])) for i in range(len(rr))]
    assert tbls.verify_beacons(pk, pr, rr, ps, bad, seed=37).tolist() == want
    dev = torch.device("cuda", 0)
    p_, r_, psb, off = tbls._beacon_arrays(pr, rr, ps)
    d_pr = torch.from_numpy(p_.astype(np.int64)).to(dev)
    d_r = torch.from_numpy(r_.astype(np.int64)).to(dev)
    d_ps = torch.from_numpy(psb).to(dev)
    d_off = torch.from_numpy(off.astype(np.int32)).to(dev)
    n = len(rr)
    lib = L.lib()
    outs = []
    for k in range(4):
        d_sig = torch.from_numpy(np.ascontiguousarray(bad if k == 2 else sigs)).to(dev)
        d_st = torch.full((n,), 99, dtype=torch.uint8, device=dev)
        torch.cuda.synchronize()
        L.check(lib.dg_verify_beacons_dev_async(L.ptr(pk), n, L.ptr(d_pr), L.ptr(d_r), L.ptr(d_ps), L.ptr(d_off),
                                                L.ptr(d_sig), L.ptr(d_st), 40 + k, None, None))
        sp = ctypes.c_void_p()
        L.check(lib.dg_last_batch_stream(ctypes.byref(sp)))
        gs = torch.cuda.ExternalStream(sp.value, device=dev)
        with torch.cuda.stream(gs):
            bits = shard.pack_bits(d_st)
            st_copy = d_st.clone()
        outs.append((k, bits, st_copy, d_sig, d_st))  # (the batch writes d_sig's statuses into d_st until done)
    L.check(lib.dg_wait_all())
    torch.cuda.synchronize()
    for k, bits, st_copy, _, _ in outs:
        got = st_copy.cpu().numpy()
        exp = np.array(want if k == 2 else [0] * n, np.uint8)
        assert np.array_equal(got, exp), k
        assert np.array_equal(bits.cpu().numpy(), np.packbits(exp != 0, bitorder="little")), k


_QUEUE_CHILD = r"""
import sys
import numpy as np
sys.path.insert(0, sys.argv[1])
from drand_amd import _lib as L
from drand_amd import tbls
from tests.fixtures import chain, chain_arrays, hx
c = chain()
pr, rr, ps, sigs, msgs = chain_arrays(c)
bad = sigs.copy()
bad[2] = sigs[3]
bad[6, 0] ^= 0x20
st = tbls.verify_beacons(hx(c["pk"]), pr, rr, ps, bad, seed=41)
np.save(sys.argv[2], st)
print(L.hw_queues())
"""


@pytest.mark.parametrize("queues", ["8", "16"])
def test_dg_init_and_per_item_pass_at_other_queue_counts(tmp_path, queues):
    """A process started with GPU_MAX_HW_QUEUES = 8 or 16 (child process: HIP reads it once) initialises -- round 4's
    first plan put the per-item kernels' scratch on every set queue and failed dg_init at 8 queues with
    HSA_STATUS_ERROR_OUT_OF_RESOURCES -- and a batch with two bad beacons gets the twin's statuses (the per-item pass on
    the dedicated stream, dg_queue_plan)."""
    out = tmp_path / "st.npy"
    r = subprocess.run([sys.executable, "-c", _QUEUE_CHILD, ROOT, str(out)],
                       env=dict(os.environ, GPU_MAX_HW_QUEUES=queues), capture_output=True, text=True, timeout=300,
                       cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    assert r.stdout.strip().splitlines()[-1] == queues
    c = chain()
    pr, rr, ps, sigs, msgs = chain_arrays(c)
    bad = sigs.copy()
    bad[2] = sigs[3]
    bad[6, 0] ^= 0x20
    pk = hx(c["pk"])
    want = [twin.verify(pk, bytes(msgs[i]), bytes(bad[i])) for i in range(len(rr))]
    assert np.load(out).tolist() == want and sum(1 for w in want if w) == 2
