"""Bulk consumers of the verification path: the callers either side of it that SURVEY.md §8(f) ranks
next, as host code over the C-ABI (what the Go side would do through the gpu/ package).

* `Beacon`            beacon.Beacon (beacon/chain.go:16-44) with its JSON store encoding (Marshal /
                      Unmarshal = encoding/json of the struct: []byte fields as standard base64) and the
                      BoltDB key roundToBytes (beacon/store.go:248-252).
* `sync_from`         beacon.Handler.syncFrom (beacon/beacon.go:529-607): replies are buffered into
                      batches of K rounds; links (A13) and signatures (A1 + A3) are checked for the whole
                      batch on the GPU, then the prefix before the first failure is stored -- the
                      reference's one-at-a-time stop-at-first-failure semantics, in bulk.
* `audit_chain`       a stored-chain audit over the store cursor (beacon/store.go:165-224): every stored
                      beacon re-verified, linked to the one before it, its randomness derived (A2).
* `verify_public_rand` core.Client.verify (core/client_public.go:107-127) for many fetched rounds.

Verdicts come from the GPU (drand_amd.tbls -> libdrandgpu.so); `verify` / `links` may be replaced by a
caller-supplied function with the same signature (the CPU tests pass the oracle's).
"""
import base64
import json
import struct
from dataclasses import dataclass
from typing import Callable, Iterable, List, Optional, Sequence, Tuple

import numpy as np

from . import _lib as L

# per-item codes beyond the DG_ST_* verdicts (include/drand_gpu.h)
ST_OK = L.ST_OK
ST_BROKEN_LINK = 6      # round not after the previous one, or prev round / prev sig do not match it
ST_NO_RANDOMNESS = 7    # client: "drand: no randomness found"
ST_BAD_RANDOMNESS = 8   # client: randomness != SHA-256(signature)
ST_BAD_RECORD = 9       # store: value does not unmarshal, or its round differs from its key


@dataclass
class Beacon:
    """beacon.Beacon (beacon/chain.go:16-28): field order as declared, which is the JSON key order."""
    previous_round: int
    previous_sig: bytes
    round: int
    signature: bytes

    def randomness(self) -> bytes:
        """RandomnessFromSignature (beacon/chain.go:52-55) -- host SHA-256 for one beacon."""
        import hashlib

        return hashlib.sha256(self.signature).digest()

    def marshal(self) -> bytes:
        """json.Marshal(b) (beacon/chain.go:38-40): compact, []byte as std base64, nil as null."""
        def b64(x):
            return None if x is None else base64.b64encode(x).decode()

        d = {"PreviousRound": int(self.previous_round), "PreviousSig": b64(self.previous_sig),
             "Round": int(self.round), "Signature": b64(self.signature)}
        return json.dumps(d, separators=(",", ":")).encode()

    @staticmethod
    def unmarshal(buf: bytes) -> "Beacon":
        """json.Unmarshal (beacon/chain.go:42-44); raises ValueError on a malformed record."""
        d = json.loads(buf)
        if not isinstance(d, dict):
            raise ValueError("beacon record is not a JSON object")

        def u64(k):
            v = d.get(k, 0)
            if not isinstance(v, int) or isinstance(v, bool) or not 0 <= v < 1 << 64:
                raise ValueError("%s is not a uint64" % k)
            return v

        def raw(k):
            v = d.get(k)
            if v is None:
                return b""
            if not isinstance(v, str):
                raise ValueError("%s is not a base64 string" % k)
            return base64.b64decode(v, validate=True)

        return Beacon(u64("PreviousRound"), raw("PreviousSig"), u64("Round"), raw("Signature"))


def round_to_bytes(r: int) -> bytes:
    """roundToBytes (beacon/store.go:248-252): the BoltDB key, big-endian uint64."""
    return struct.pack(">Q", r)


def _gpu_verify(pub: bytes, prev_rounds, rounds, prev_sigs, sigs) -> np.ndarray:
    from . import tbls

    return tbls.verify_beacons(pub, prev_rounds, rounds, prev_sigs, sigs)


def _gpu_links(cur_round, cur_sig, prev_rounds, rounds, prev_sigs, sigs) -> np.ndarray:
    from . import tbls

    return tbls.check_links(cur_round, cur_sig, prev_rounds, rounds, prev_sigs, sigs)


def _gpu_randomness(sigs) -> np.ndarray:
    from . import tbls

    return tbls.randomness(sigs)


def _sig_block(beacons: Sequence[Beacon]) -> np.ndarray:
    """(n, 96) signatures; a signature that is not 96 B becomes 96 zero bytes, which does not decode
    (no compression flag), so its verdict is the reference's decode error."""
    out = np.zeros((len(beacons), 96), np.uint8)
    for i, b in enumerate(beacons):
        if len(b.signature) == 96:
            out[i] = np.frombuffer(b.signature, np.uint8)
    return out


def _verify_block(pub, beacons, verify) -> np.ndarray:
    st = np.asarray(verify(pub, [b.previous_round for b in beacons], [b.round for b in beacons],
                           [b.previous_sig for b in beacons], _sig_block(beacons)), dtype=np.uint8).copy()
    for i, b in enumerate(beacons):
        if len(b.signature) != 96 and st[i] == ST_OK:
            st[i] = L.ST_SIG_DECODE
    return st


@dataclass
class SyncResult:
    last: Optional[Beacon]      # currentBeacon of syncFrom: the last beacon stored, None if none
    round: int                  # currentRound at return
    stored: int                 # beacons passed to `put`
    error: Optional[str]        # nil / non-nil as syncFrom's error


def sync_from(pub: bytes, init_round: int, init_sig: bytes, peers: Iterable[Iterable[Beacon]],
              put: Optional[Callable[[Beacon], None]] = None, next_round: Optional[int] = None,
              batch: int = 16384, verify: Callable = _gpu_verify, links: Callable = _gpu_links) -> SyncResult:
    """beacon.Handler.syncFrom (beacon/beacon.go:529-607) over the reply streams of the peers in order.

    Per peer, replies are taken `batch` at a time.  A reply is accepted iff (as the reference checks it
    one by one) its round is above the current round, its previous round / signature are the current
    ones (beacon.go:561-573), and VerifyRecovered(pub, Message(prevSig, prevRound, round), sig) holds
    (beacon.go:575).  Accepted replies are stored in order; the first failing reply ends this peer's
    stream (the reference cancels it and moves to the next peer).  `next_round` stands for NextRound of
    the group clock: once the current round reaches next_round - 1 the sync is done (beacon.go:594-601).
    Links are checked on the GPU against the previous reply of the batch (dg_check_links), signatures
    for the whole batch at once (dg_verify_beacons: one RLC multi-pairing)."""
    cur_round, cur_sig = int(init_round), bytes(init_sig)
    last, stored = None, 0
    for stream in peers:
        it = iter(stream)
        alive = True
        while alive:
            chunk: List[Beacon] = []
            for b in it:
                chunk.append(b)
                if len(chunk) == batch:
                    break
            if not chunk:
                break
            ln = np.asarray(links(cur_round, cur_sig, [b.previous_round for b in chunk], [b.round for b in chunk],
                                  [b.previous_sig for b in chunk], _sig_block(chunk)), dtype=np.uint8)
            st = _verify_block(pub, chunk, verify)
            bad = np.nonzero((ln != 0) | (st != 0))[0]
            good = int(bad[0]) if len(bad) else len(chunk)
            for b in chunk[:good]:
                if put is not None:
                    put(b)
                stored += 1
                last, cur_round, cur_sig = b, int(b.round), bytes(b.signature)
                if next_round is not None and cur_round + 1 == next_round:
                    return SyncResult(last, cur_round, stored, None)
            if good < len(chunk):
                alive = False  # cancel(): this peer's stream ends at its first bad reply
    err = "syncing went from %d to %d whereas current round is %s: network is down" % (
        init_round, cur_round, (next_round - 1) if next_round is not None else "unknown")
    return SyncResult(last, cur_round, stored, err)


@dataclass
class AuditReport:
    rounds: np.ndarray          # round of every record (0 where the record did not unmarshal)
    status: np.ndarray          # per record: 0 ok, DG_ST_* verdict, ST_BROKEN_LINK, ST_BAD_RECORD
    randomness: np.ndarray      # (n, 32) SHA-256 of each signature (zeros for unusable records)

    @property
    def ok(self) -> bool:
        return not self.status.any()


def audit_chain(pub: bytes, records: Iterable[Tuple[bytes, bytes]], batch: int = 100000,
                verify: Callable = _gpu_verify, randomness: Callable = _gpu_randomness) -> AuditReport:
    """Stored-chain audit: walk the store cursor (beacon/store.go:165-224; records = (key, value) pairs
    in key order, value = Beacon.Marshal) and check every record: it unmarshals and its round equals
    its key (roundToBytes), it links to the record before it (previous round and signature, as
    syncFrom checks a fresh reply), and VerifyBeacon holds (beacon/chain.go:65-71).  The first record
    is not link-checked (the audit may start mid-chain, as Cursor.Seek does).  Signatures are verified
    `batch` records per GPU call, randomness (A2) derived on the GPU."""
    beacons: List[Optional[Beacon]] = []
    for k, v in records:
        try:
            b = Beacon.unmarshal(v)
            if bytes(k) != round_to_bytes(b.round):
                b = None
        except (ValueError, json.JSONDecodeError):
            b = None
        beacons.append(b)
    n = len(beacons)
    status = np.zeros(n, np.uint8)
    rounds = np.array([b.round if b is not None else 0 for b in beacons], np.uint64)
    rand = np.zeros((n, 32), np.uint8)
    idx = [i for i, b in enumerate(beacons) if b is not None]
    for i, b in enumerate(beacons):
        if b is None:
            status[i] = ST_BAD_RECORD
    for s in range(0, len(idx), batch):
        part = idx[s:s + batch]
        blk = [beacons[i] for i in part]
        st = _verify_block(pub, blk, verify)
        status[part] = st
        sigs = _sig_block(blk)
        rand[part] = np.asarray(randomness(sigs), np.uint8).reshape(-1, 32)
        for j, i in enumerate(part):
            if len(blk[j].signature) != 96:
                rand[i] = 0
    for i in range(1, n):
        b, p = beacons[i], beacons[i - 1]
        if b is None or p is None or status[i] != ST_OK:
            continue
        if not (b.round > p.round and b.previous_round == p.round and b.previous_sig == p.signature):
            status[i] = ST_BROKEN_LINK
    return AuditReport(rounds, status, rand)


@dataclass
class PublicRand:
    """drand.PublicRandResponse (protobuf/drand/api.proto): the fields core.Client.verify reads."""
    previous_signature: bytes
    previous_round: int
    round: int
    signature: bytes
    randomness: Optional[bytes]


def verify_public_rand(pub: bytes, responses: Sequence[PublicRand], verify: Callable = _gpu_verify,
                       randomness: Callable = _gpu_randomness) -> np.ndarray:
    """core.Client.verify (core/client_public.go:107-127) for many responses: per response 0 (nil),
    ST_NO_RANDOMNESS (randomness missing or empty -- checked first, as the reference does), the VerifyRecovered
    verdict, or ST_BAD_RANDOMNESS (randomness != SHA-256(signature))."""
    n = len(responses)
    out = np.zeros(n, np.uint8)
    beacons = [Beacon(r.previous_round, r.previous_signature, r.round, r.signature) for r in responses]
    if n == 0:
        return out
    st = _verify_block(pub, beacons, verify)
    rand = np.asarray(randomness(_sig_block(beacons)), np.uint8).reshape(-1, 32)
    for i, r in enumerate(responses):
        if not r.randomness:  # proto3: an empty bytes field arrives as nil
            out[i] = ST_NO_RANDOMNESS
        elif st[i] != ST_OK:
            out[i] = st[i]
        elif bytes(rand[i]) != bytes(r.randomness):
            out[i] = ST_BAD_RANDOMNESS
    return out
