"""Threshold-BLS (kyber sign/tbls + sign/bls + share) and drand beacon helpers -- TEST INFRASTRUCTURE ONLY.

Restatement of the semantics drand relies on through `key.Scheme` (key/curve.go:30,
`tbls.NewThresholdSchemeOnG2(Pairing)`); the kyber module itself is not in the container
(github.com/drand/kyber @ v1.0.1-0.20200331114745-30e90cc60f99, go.mod:10), so the rules below
follow SURVEY.md §8(a) rows A1-A14:

  A1  beacon.Message            beacon/chain.go:86-94, roundToBytes beacon/store.go:248-252
  A2  RandomnessFromSignature   beacon/chain.go:52-55
  A4  VerifyRecovered = bls.Verify: e(X, H(m)) == e(g1, sigma)
  A5  VerifyPartial: i = BE16(sig[:2]); bls.Verify(PubPoly.Eval(i), msg, sig[2:])
  A6  Recover: first t valid partials in input order, dedupe by index (xyCommit),
      Lagrange at 0 over x = i+1, error if < t distinct
  A7  Sign: BE16(i) || compress(x_i * H(m))
  A12 PubPoly.Eval: Horner over the G1 commits at x = i+1
  A13 chain link check  beacon/beacon.go:561-573
"""
import hashlib

from . import bls12381 as B

# status codes of the C-ABI (include/drand_gpu.h)
ST_OK = 0
ST_BAD_SIG = 1      # pairing check failed
ST_SIG_DECODE = 2   # sigma does not decode (flags, non-canonical, off-curve, off-subgroup)
ST_BAD_INDEX = 3    # partial too short / index parse
ST_PK_DECODE = 4
ST_NOT_ENOUGH = 5   # Recover: fewer than t distinct good shares


class TblsError(Exception):
    def __init__(self, status, msg=""):
        super().__init__(msg or "status %d" % status)
        self.status = status


def round_to_bytes(r):
    return int(r).to_bytes(8, "big")


def beacon_message(prev_sig, prev_round, cur_round):
    """beacon/chain.go:86-94 -- SHA256(BE64(prevRound) || prevSig || BE64(round))."""
    return hashlib.sha256(round_to_bytes(prev_round) + bytes(prev_sig) + round_to_bytes(cur_round)).digest()


def randomness(sig):
    """beacon/chain.go:52-55."""
    return hashlib.sha256(bytes(sig)).digest()


# ----------------------------------------------------------------------------- polynomials (kyber share)
class PriPoly:
    def __init__(self, coeffs):
        self.coeffs = [c % B.R for c in coeffs]

    def eval(self, i):
        x = i + 1
        acc = 0
        for c in reversed(self.coeffs):
            acc = (acc * x + c) % B.R
        return acc

    def shares(self, n):
        return [(i, self.eval(i)) for i in range(n)]

    def secret(self):
        return self.coeffs[0]

    def commit(self):
        return [B.G1C.mul(B.G1_GEN, c) for c in self.coeffs]


def _points(commits):
    return [B.g1_decompress(bytes(c)) if isinstance(c, (bytes, bytearray)) else c for c in commits]


def pubpoly_eval(commits, i):
    """Horner in G1 at x = i+1 (kyber share.PubPoly.Eval); commits as points or 48 B encodings."""
    commits = _points(commits)
    x = i + 1
    acc = None
    for c in reversed(commits):
        acc = B.G1C.add(B.G1C.mul(acc, x), c)
    return acc


# ----------------------------------------------------------------------------- bls / tbls
def bls_sign(x, msg):
    return B.g2_compress(B.G2C.mul(B.hash_to_g2(msg), x))


def bls_verify_status(pk_point, msg, sig96):
    """Status of bls.Verify(pk, msg, sig) with the error taxonomy of include/drand_gpu.h."""
    try:
        s = B.g2_decompress(bytes(sig96))
    except B.DecodeError:
        return ST_SIG_DECODE
    h = B.hash_to_g2(msg)
    ok = B.pairing_check([(pk_point, h), (B.G1C.neg(B.G1_GEN), s)])
    return ST_OK if ok else ST_BAD_SIG


def tbls_sign(share, msg):
    i, v = share
    return int(i).to_bytes(2, "big") + bls_sign(v, msg)


def index_of(sig):
    if len(sig) < 2:
        raise TblsError(ST_BAD_INDEX, "invalid signature share")
    return int.from_bytes(bytes(sig[:2]), "big")


def verify_partial_status(commits, msg, sig):
    try:
        i = index_of(sig)
    except TblsError:
        return ST_BAD_INDEX
    if len(sig) != 98:
        return ST_SIG_DECODE
    return bls_verify_status(pubpoly_eval(commits, i), msg, bytes(sig[2:]))


def lagrange_at_zero(indices):
    xs = [i + 1 for i in indices]
    lams = []
    for a, xi in enumerate(xs):
        num, den = 1, 1
        for b, xj in enumerate(xs):
            if a != b:
                num = num * xj % B.R
                den = den * (xj - xi) % B.R
        lams.append(num * pow(den, B.R - 2, B.R) % B.R)
    return lams


def recover(commits, msg, sigs, t, n, statuses=None):
    """tbls.Recover semantics.  Returns (sig96 or None, round_status, share_statuses).

    share_statuses[k] is the VerifyPartial status of sigs[k] for every partial Recover looked at, and
    255 for the partials after the t-th collected one (never examined, like the reference's early break).
    """
    if statuses is None:
        statuses = [None] * len(sigs)
    share_status = [255] * len(sigs)
    collected = []
    for k, sig in enumerate(sigs):
        st = statuses[k] if statuses[k] is not None else verify_partial_status(commits, msg, sig)
        share_status[k] = st
        if st != ST_OK:
            continue
        collected.append((index_of(sig), B.g2_decompress(bytes(sig[2:]))))
        if len(collected) >= t:
            break
    distinct = {}
    for i, pt in sorted(collected, key=lambda x: x[0]):
        if len(distinct) == t:
            break
        distinct[i] = pt
    if len(distinct) < t:
        return None, ST_NOT_ENOUGH, share_status
    idx = sorted(distinct)
    lams = lagrange_at_zero(idx)
    acc = None
    for i, lam in zip(idx, lams):
        acc = B.G2C.add(acc, B.G2C.mul(distinct[i], lam))
    return B.g2_compress(acc), ST_OK, share_status


def check_links(cur_round, cur_sig, prev_rounds, rounds, prev_sigs, sigs):
    """beacon/beacon.go:561-573 per item: reply.Round > cur && prevRound == cur && prevSig == curSig."""
    out = []
    for k in range(len(rounds)):
        ok = rounds[k] > cur_round and prev_rounds[k] == cur_round and bytes(prev_sigs[k]) == bytes(cur_sig)
        out.append(0 if ok else 1)
        cur_round, cur_sig = rounds[k], sigs[k]
    return out
