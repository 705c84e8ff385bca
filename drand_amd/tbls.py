"""Host-side mirror of kyber's `sign.ThresholdScheme` as drand uses it through `key.Scheme`.

Reference interface (the kyber module is not vendored; signatures per SURVEY.md §8(b)):
    key/curve.go:30        var Scheme = tbls.NewThresholdSchemeOnG2(Pairing)
    Sign(*share.PriShare, msg) ([]byte, error)                 beacon/beacon.go:433
    IndexOf(sig []byte) (int, error)                            beacon/beacon.go:154, round_cache.go:113
    VerifyPartial(*share.PubPoly, msg, sig []byte) error        beacon/beacon.go:148
    VerifyRecovered(kyber.Point, msg, sig []byte) error         beacon/beacon.go:494,575; chain.go:70
    Recover(*share.PubPoly, msg, sigs [][]byte, t, n) ([]byte, error)   beacon/beacon.go:488

Same names, same argument meaning, same error behaviour (an exception where kyber returns a non-nil
error; error *text* is not reproduced).  Every method runs on the MI355X through libdrandgpu.so; the
batch methods are the data-parallel extensions the GPU exists for.  Points cross as kyber bytes:
48 B G1, 96 B G2, partials = BE16(index) || 96 B G2.
"""
from dataclasses import dataclass
from typing import List, Sequence

import numpy as np

from . import _lib as L

R_ORDER = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001


class SchemeError(Exception):
    """Non-nil kyber error.  `status` is the DG_ST_* code of the failing item."""

    def __init__(self, status, what=""):
        super().__init__("%s (status %d)" % (what or "threshold scheme error", status))
        self.status = status


@dataclass
class PriShare:
    """kyber share.PriShare: index I (x = I + 1) and value V (a scalar mod r)."""

    I: int
    V: int


@dataclass
class PubPoly:
    """kyber share.PubPoly: commitments (48 B compressed G1) of a degree t-1 polynomial."""

    commits: List[bytes]

    @property
    def threshold(self):
        return len(self.commits)

    def commit(self):
        """PubPoly.Commit(): the constant term, i.e. the group public key (key/keys.go:258-260)."""
        return self.commits[0]

    def eval(self, i):
        """PubPoly.Eval(i).V, on the GPU."""
        return pubpoly_eval(self, [i])[0]

    def commits_array(self):
        return L.u8(self.commits, (len(self.commits), 48))


def _msgs_array(msgs):
    if isinstance(msgs, np.ndarray):
        arr = np.ascontiguousarray(msgs, dtype=np.uint8)
        return arr.reshape(arr.shape[0], -1)
    lens = {len(m) for m in msgs}
    if len(lens) != 1:
        raise ValueError("all messages of one batch must have the same length")
    return L.u8(msgs, (len(msgs), lens.pop()))


def hash_to_g2(msgs, dst=L.DST_NUL):
    m = _msgs_array(msgs)
    n = m.shape[0]
    out = np.zeros((n, 96), dtype=np.uint8)
    L.check(L.lib().dg_hash_to_g2(n, L.ptr(m), m.shape[1], L.ptr(dst), len(dst), L.ptr(out)))
    return out


def pubpoly_eval(pub: PubPoly, indices):
    idx = np.ascontiguousarray(indices, dtype=np.uint32)
    out = np.zeros((len(idx), 48), dtype=np.uint8)
    c = pub.commits_array()
    L.check(L.lib().dg_pubpoly_eval(L.ptr(c), c.shape[0], len(idx), L.ptr(idx), L.ptr(out)))
    return [bytes(r) for r in out]


def sign_batch(scalars: Sequence[int], msgs, indices=None):
    """Batch tbls.Sign (indices given) or bls.Sign (indices None) on the GPU."""
    m = _msgs_array(msgs)
    n = m.shape[0]
    sc = L.u8([int(s % R_ORDER).to_bytes(32, "big") for s in scalars], (n, 32))
    if indices is None:
        out = np.zeros((n, 96), dtype=np.uint8)
        L.check(L.lib().dg_sign(n, L.ptr(sc), None, L.ptr(m), m.shape[1], L.ptr(out)))
    else:
        idx = np.ascontiguousarray(indices, dtype=np.uint16)
        out = np.zeros((n, 98), dtype=np.uint8)
        L.check(L.lib().dg_sign(n, L.ptr(sc), L.ptr(idx), L.ptr(m), m.shape[1], L.ptr(out)))
    return out


def verify_recovered_batch(public: bytes, msgs, sigs, seed=0):
    """Per-item bls.Verify statuses (DG_ST_*) of a batch against one key."""
    m = _msgs_array(msgs)
    n = m.shape[0]
    s = L.u8(sigs, (n, 96))
    st = np.zeros(n, dtype=np.uint8)
    L.check(L.lib().dg_verify(L.ptr(bytes(public)), n, L.ptr(m), m.shape[1], L.ptr(s), L.ptr(st), seed))
    return st


def verify_partial_batch(pub: PubPoly, msgs, partials, seed=0):
    """msgs: R messages; partials: (R, k, 98) -> statuses (R, k)."""
    m = _msgs_array(msgs)
    R = m.shape[0]
    p = L.u8(partials)
    p = p.reshape(R, -1, 98)
    k = p.shape[1]
    st = np.zeros((R, k), dtype=np.uint8)
    c = pub.commits_array()
    L.check(L.lib().dg_verify_partials(L.ptr(c), c.shape[0], R, L.ptr(m), m.shape[1], k, L.ptr(p), L.ptr(st), seed))
    return st


def recover_batch(pub: PubPoly, msgs, partials, t, n, seed=0):
    """msgs: R messages; partials: (R, k, 98).  Returns (sigs (R, 96), round_status (R,), share_status (R, k))."""
    m = _msgs_array(msgs)
    R = m.shape[0]
    p = L.u8(partials).reshape(R, -1, 98)
    k = p.shape[1]
    out = np.zeros((R, 96), dtype=np.uint8)
    rs = np.zeros(R, dtype=np.uint8)
    ss = np.zeros((R, k), dtype=np.uint8)
    c = pub.commits_array()
    L.check(L.lib().dg_recover(L.ptr(c), c.shape[0], n, R, L.ptr(m), m.shape[1], k, L.ptr(p), L.ptr(out), L.ptr(rs),
                               L.ptr(ss), seed))
    return out, rs, ss


def recover_batch_dev(pub: PubPoly, d_msgs, d_partials, t, n, seed=0):
    """recover_batch with device-resident inputs and outputs (dg_recover_dev): d_msgs a (R, msg_len) and
    d_partials a (R, k, 98) uint8 torch tensor on the current GPU.  Returns device tensors (sigs (R, 96),
    round_status (R,), share_status (R, k))."""
    import torch

    R, k = d_partials.shape[0], d_partials.shape[1]
    dev = d_partials.device
    out = torch.empty((R, 96), dtype=torch.uint8, device=dev)
    rs = torch.empty(R, dtype=torch.uint8, device=dev)
    ss = torch.empty((R, k), dtype=torch.uint8, device=dev)
    c = pub.commits_array()
    torch.cuda.current_stream(dev).synchronize()  # inputs written on torch's stream are visible to the library's
    L.check(L.lib().dg_recover_dev(L.ptr(c), c.shape[0], n, R, L.ptr(d_msgs), d_msgs.shape[1], k, L.ptr(d_partials),
                                   L.ptr(out), L.ptr(rs), L.ptr(ss), seed))
    return out, rs, ss


def verify_partial_batch_dev(pub: PubPoly, d_msgs, d_partials, seed=0):
    """verify_partial_batch with device-resident inputs and output (dg_verify_partials_dev): d_msgs (R, msg_len),
    d_partials (R, k, 98) uint8 torch tensors on the current GPU -> statuses (R, k) device tensor."""
    import torch

    R, k = d_partials.shape[0], d_partials.shape[1]
    st = torch.empty((R, k), dtype=torch.uint8, device=d_partials.device)
    c = pub.commits_array()
    torch.cuda.current_stream(d_partials.device).synchronize()
    L.check(L.lib().dg_verify_partials_dev(L.ptr(c), c.shape[0], R, L.ptr(d_msgs), d_msgs.shape[1], k,
                                           L.ptr(d_partials), L.ptr(st), seed))
    return st


def recover_verified_batch_dev(d_partials, d_verified_status, t, n):
    """recover_verified_batch with device-resident partials (R, k, 98), verdicts (R, k) and outputs
    (dg_recover_verified_dev) -> device tensors (sigs (R, 96), round_status (R,), share_status (R, k))."""
    import torch

    R, k = d_partials.shape[0], d_partials.shape[1]
    dev = d_partials.device
    out = torch.empty((R, 96), dtype=torch.uint8, device=dev)
    rs = torch.empty(R, dtype=torch.uint8, device=dev)
    ss = torch.empty((R, k), dtype=torch.uint8, device=dev)
    torch.cuda.current_stream(dev).synchronize()
    L.check(L.lib().dg_recover_verified_dev(t, n, R, k, L.ptr(d_partials), L.ptr(d_verified_status), L.ptr(out),
                                            L.ptr(rs), L.ptr(ss)))
    return out, rs, ss


def recover_verified_batch(pub: PubPoly, msgs, partials, verified_status, t, n):
    """The live round's Recover (beacon/beacon.go:472-494) with the VerifyPartial verdicts ProcessBeacon
    already holds (beacon/beacon.go:148): partials (R, k, 98), verified_status (R, k) DG_ST_* ->
    (sigs (R, 96), round_status (R,), share_status (R, k)); no pairing is recomputed.  `pub` and `msgs`
    are what kyber's Recover takes; the verdicts stand in for the re-verification they would feed."""
    del pub, msgs  # only the re-verification reads them
    p = L.u8(partials)
    st_in = np.ascontiguousarray(verified_status, dtype=np.uint8)
    R = st_in.shape[0]
    p = p.reshape(R, -1, 98)
    k = p.shape[1]
    out = np.zeros((R, 96), dtype=np.uint8)
    rs = np.zeros(R, dtype=np.uint8)
    ss = np.zeros((R, k), dtype=np.uint8)
    L.check(L.lib().dg_recover_verified(t, n, R, k, L.ptr(p), L.ptr(st_in), L.ptr(out), L.ptr(rs), L.ptr(ss)))
    return out, rs, ss


def set_hash_dst(dst=None):
    """Switch the hash-to-G2 DST of every sign / verify / recover entry point (None: the NUL default)."""
    d = b"" if dst is None else bytes(dst)
    L.check(L.lib().dg_set_hash_dst(L.ptr(d) if d else None, len(d)))


def hash_dst():
    import ctypes

    buf = np.zeros(256, np.uint8)
    n = ctypes.c_size_t()
    L.check(L.lib().dg_get_hash_dst(L.ptr(buf), 256, ctypes.cast(ctypes.pointer(n), ctypes.c_void_p)))
    return bytes(buf[:n.value])


def _beacon_arrays(prev_rounds, rounds, prev_sigs):
    pr = np.ascontiguousarray(prev_rounds, dtype=np.uint64)
    rr = np.ascontiguousarray(rounds, dtype=np.uint64)
    ps = [bytes(x) for x in prev_sigs]
    off = np.zeros(len(ps) + 1, dtype=np.uint32)
    off[1:] = np.cumsum([len(x) for x in ps])
    psb = L.u8(ps) if ps else np.zeros(0, np.uint8)
    return pr, rr, psb, off


def verify_beacons(public: bytes, prev_rounds, rounds, prev_sigs, sigs, seed=0):
    """beacon.VerifyBeacon (beacon/chain.go:65-71) over a batch: statuses (DG_ST_*) per beacon."""
    pr, rr, psb, off = _beacon_arrays(prev_rounds, rounds, prev_sigs)
    n = len(rr)
    s = L.u8(sigs, (n, 96))
    st = np.zeros(n, dtype=np.uint8)
    L.check(L.lib().dg_verify_beacons(L.ptr(bytes(public)), n, L.ptr(pr), L.ptr(rr), L.ptr(psb), L.ptr(off), L.ptr(s),
                                      L.ptr(st), seed))
    return st


def beacon_messages(prev_rounds, rounds, prev_sigs):
    """beacon.Message (beacon/chain.go:86-94) batch -> (n, 32)."""
    pr, rr, psb, off = _beacon_arrays(prev_rounds, rounds, prev_sigs)
    out = np.zeros((len(rr), 32), dtype=np.uint8)
    L.check(L.lib().dg_beacon_messages(len(rr), L.ptr(pr), L.ptr(rr), L.ptr(psb), L.ptr(off), L.ptr(out)))
    return out


def randomness(sigs):
    """beacon.RandomnessFromSignature (beacon/chain.go:52-55) batch -> (n, 32)."""
    s = L.u8(sigs)
    s = s.reshape(-1, 96)
    out = np.zeros((s.shape[0], 32), dtype=np.uint8)
    L.check(L.lib().dg_randomness(s.shape[0], L.ptr(s), L.ptr(out)))
    return out


def check_links(cur_round, cur_sig, prev_rounds, rounds, prev_sigs, sigs):
    """syncFrom's link check (beacon/beacon.go:561-573): 0 linked / 1 broken per beacon."""
    pr, rr, psb, off = _beacon_arrays(prev_rounds, rounds, prev_sigs)
    n = len(rr)
    s = L.u8(sigs, (n, 96))
    out = np.zeros(n, dtype=np.uint8)
    cs = bytes(cur_sig)
    L.check(L.lib().dg_check_links(int(cur_round), L.ptr(cs), len(cs), n, L.ptr(pr), L.ptr(rr), L.ptr(psb), L.ptr(off),
                                   L.ptr(s), L.ptr(out)))
    return out


class ThresholdScheme:
    """`tbls.NewThresholdSchemeOnG2(bls12381)`: keys on G1, signatures on G2 (key/curve.go:21-30)."""

    def sign(self, private: PriShare, msg: bytes) -> bytes:
        return bytes(sign_batch([private.V], [bytes(msg)], [private.I])[0])

    def index_of(self, sig: bytes) -> int:
        if len(sig) < 2:
            raise SchemeError(L.ST_BAD_INDEX, "invalid signature share")
        return int.from_bytes(bytes(sig[:2]), "big")

    def verify_partial(self, public: PubPoly, msg: bytes, sig: bytes) -> None:
        if len(sig) < 2:
            raise SchemeError(L.ST_BAD_INDEX, "invalid signature share")
        if len(sig) != 98:
            raise SchemeError(L.ST_SIG_DECODE, "signature share has the wrong length")
        st = int(verify_partial_batch(public, [bytes(msg)], [bytes(sig)])[0, 0])
        if st != L.ST_OK:
            raise SchemeError(st, "partial signature invalid")

    def verify_recovered(self, public: bytes, msg: bytes, sig: bytes) -> None:
        if len(sig) != 96:
            raise SchemeError(L.ST_SIG_DECODE, "signature has the wrong length")
        st = int(verify_recovered_batch(public, [bytes(msg)], [bytes(sig)])[0])
        if st != L.ST_OK:
            raise SchemeError(st, "signature invalid")

    def recover(self, public: PubPoly, msg: bytes, sigs: Sequence[bytes], t: int, n: int) -> bytes:
        # fixed-size records cross the C-ABI; shorter/longer partials can never verify, kyber skips them
        good = [bytes(s) for s in sigs if len(s) == 98]
        if len(good) == 0:
            raise SchemeError(L.ST_NOT_ENOUGH, "not enough valid partials")
        out, rs, _ = recover_batch(public, [bytes(msg)], [good], t, n)
        if int(rs[0]) != L.ST_OK:
            raise SchemeError(int(rs[0]), "not enough valid partials")
        return bytes(out[0])


Scheme = ThresholdScheme()
