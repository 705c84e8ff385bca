"""Round-3 parity tests of the HIP path through the C-ABI: Recover's examined-prefix window (drand_gpu.hip
recover_windowed).  The batch equation covers each round's first t partials only -- kyber's tbls.Recover verifies
partials in input order and stops at the t-th valid one (beacon/beacon.go:488) -- and the partials beyond the
window are decoded and checked only when a round's window did not yield t valid shares.  Every case is compared
with the CPU twin's Recover (signatures, round statuses, every share status).  Bit-exact throughout."""
import hashlib

import numpy as np
import pytest

from drand_amd import _lib as L
from drand_amd import tbls
from oracle import twin
from tests.fixtures import group

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def device():
    L.lib(0)
    yield


def _rounds(t, n, R, label, shuffle=True):
    coeffs, commits, shares = group(t, n)
    msgs = [hashlib.sha256(b"%s/%d" % (label, r)).digest() for r in range(R)]
    sc = [v for _ in range(R) for _, v in shares]
    idx = [i for _ in range(R) for i, _ in shares]
    parts = tbls.sign_batch(sc, [m for m in msgs for _ in range(n)], idx).reshape(R, n, 98)
    if shuffle:  # a different index order per round: the window's key slots differ from the whole batch's
        rng = np.random.default_rng(int.from_bytes(hashlib.sha256(label).digest()[:4], "big"))
        for r in range(R):
            parts[r] = parts[r][rng.permutation(n)]
    return coeffs, commits, msgs, parts


def _vs_twin(commits, t, n, msgs, parts, seed):
    pub = tbls.PubPoly(commits)
    sigs, rs, ss = tbls.recover_batch(pub, msgs, parts, t, n, seed=seed)
    tw_sigs, tw_rs, tw_ss = twin.recover_batch(commits, t, n, np.array([list(m) for m in msgs], np.uint8), parts, 8)
    assert np.array_equal(rs, tw_rs)
    assert np.array_equal(ss, tw_ss)
    assert np.array_equal(sigs[rs == 0], tw_sigs[tw_rs == 0])
    return sigs, rs, ss


def test_window_clean_rounds_examine_only_t():
    """Every round valid, indices shuffled per round: the window decides, shares beyond it are not examined."""
    t, n, R = 5, 12, 40
    coeffs, commits, msgs, parts = _rounds(t, n, R, b"w-clean")
    sigs, rs, ss = _vs_twin(commits, t, n, msgs, parts, 3)
    assert not rs.any() and (ss[:, :t] == 0).all() and (ss[:, t:] == 255).all()
    for r in range(0, R, 7):
        assert bytes(sigs[r]) == twin.sign(coeffs[0], msgs[r])


def test_window_decode_failures_reach_beyond_the_window():
    """Undecodable window shares (the batch equation still holds over the rest): those rounds continue with the
    shares beyond the window, checked one by one."""
    t, n, R = 5, 12, 40
    _, commits, msgs, parts = _rounds(t, n, R, b"w-decode")
    parts[3, 1, 2:] = 0xff                   # not a field element
    parts[9, 0, 2] &= 0x7f                   # compression flag cleared
    parts[9, 4, 2:] = 0xff
    parts[17, :t, 2:] = 0xff                 # the whole window undecodable
    _, rs, ss = _vs_twin(commits, t, n, msgs, parts, 4)
    assert not rs.any()
    assert (ss[17, :t] == L.ST_SIG_DECODE).all() and (ss[17, t:2 * t] == 0).all()


def test_window_bad_signatures_and_duplicates():
    """A valid partial of another round inside a window (the batch equation fails: every examined verdict comes
    from the per-item pass), a bad share beyond the window, a duplicated index inside a window, and a round
    with fewer than t valid shares."""
    t, n, R = 5, 12, 40
    _, commits, msgs, parts = _rounds(t, n, R, b"w-bad")
    parts[2, 2] = parts[3, 2]                # another round's partial: bad signature
    parts[2, t + 1, 60] ^= 0x04              # beyond the window: examined only if needed
    parts[11, 1] = parts[11, 0]              # duplicate index among the first t valid -> not enough (xyCommit)
    parts[20, :n - t + 1, 2:] = 0xff         # n - t + 1 undecodable: fewer than t valid
    _, rs, ss = _vs_twin(commits, t, n, msgs, parts, 5)
    assert rs[11] == L.ST_NOT_ENOUGH and rs[20] == L.ST_NOT_ENOUGH
    assert ss[2, 2] == L.ST_BAD_SIG


@pytest.mark.parametrize("t,n", [(8, 8), (9, 8)])
def test_window_covers_every_share_when_t_reaches_n(t, n):
    """t >= n: the window is the whole round (t > n: never enough shares)."""
    R = 16
    _, commits, msgs, parts = _rounds(t, n, R, b"w-full%d" % t)
    _, rs, _ = _vs_twin(commits, t, n, msgs, parts, 6)
    assert (rs != 0).all() if t > n else not rs.any()


def test_window_dev_entry_equals_host_entry():
    """dg_recover_dev (HBM-resident inputs) and dg_recover give the same outputs on a mixed batch."""
    import torch

    t, n, R = 5, 12, 64
    _, commits, msgs, parts = _rounds(t, n, R, b"w-dev")
    parts[5, 0, 2:] = 0xff
    parts[6, 3] = parts[7, 3]
    pub = tbls.PubPoly(commits)
    hs, hrs, hss = tbls.recover_batch(pub, msgs, parts, t, n, seed=7)
    dev = torch.device("cuda", 0)
    d_m = torch.from_numpy(np.array([list(m) for m in msgs], np.uint8)).to(dev)
    d_p = torch.from_numpy(np.ascontiguousarray(parts)).to(dev)
    ds, drs, dss = (x.cpu().numpy() for x in tbls.recover_batch_dev(pub, d_m, d_p, t, n, seed=7))
    assert np.array_equal(hs, ds) and np.array_equal(hrs, drs) and np.array_equal(hss, dss)
