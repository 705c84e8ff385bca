"""Bulk consumers (drand_amd/bulk.py) against sequential restatements of the
reference loops: syncFrom (beacon/beacon.go:529-607), the store cursor audit (beacon/store.go:165-224)
and core.Client.verify (core/client_public.go:107-127).  The CPU tests drive the batching logic with the
CPU twin as verifier (tests only); the gpu-marked tests run the product path (libdrandgpu.so)."""
import base64
import hashlib
import json

import numpy as np
import pytest

from drand_amd import bulk
from drand_amd.bulk import Beacon, PublicRand
from oracle import twin
from tests.fixtures import chain, hx


def _status(pk, b):
    """kyber VerifyRecovered on one beacon (a signature that is not 96 B fails to unmarshal)."""
    if len(b.signature) != 96:
        return 2
    return twin.verify(pk, twin.beacon_message(b.previous_sig, b.previous_round, b.round), b.signature)


def twin_verify(pub, prev_rounds, rounds, prev_sigs, sigs):
    return np.array([twin.verify(pub, twin.beacon_message(bytes(ps), int(pr), int(r)), bytes(s))
                     for pr, r, ps, s in zip(prev_rounds, rounds, prev_sigs, sigs)], np.uint8)


def host_links(cur_round, cur_sig, prev_rounds, rounds, prev_sigs, sigs):
    out = []
    for pr, r, ps, s in zip(prev_rounds, rounds, prev_sigs, sigs):
        out.append(0 if (r > cur_round and pr == cur_round and bytes(ps) == cur_sig) else 1)
        cur_round, cur_sig = r, bytes(s)
    return np.array(out, np.uint8)


def twin_randomness(sigs):
    return np.array([list(hashlib.sha256(bytes(s)).digest()) for s in sigs], np.uint8).reshape(-1, 32)


CPU = dict(verify=twin_verify, links=host_links)


def ref_sync_from(pk, init_round, init_sig, peers, next_round=None):
    """beacon.go:529-607 one reply at a time (the oracle of the loop semantics)."""
    cur_round, cur_sig, stored = init_round, init_sig, []
    for stream in peers:
        for b in stream:
            if b.round <= cur_round:
                break
            if cur_round != b.previous_round or b.previous_sig != cur_sig:
                break
            if _status(pk, b) != 0:
                break
            stored.append(b)
            cur_round, cur_sig = b.round, b.signature
            if next_round is not None and cur_round + 1 == next_round:
                return stored, None
    return stored, "network is down"


def beacons():
    c = chain()
    return hx(c["pk"]), [Beacon(r["prev_round"], hx(r["prev_sig"]), r["round"], hx(r["sig"])) for r in c["rounds"]]


def scenarios():
    """(name, init_round, init_sig, peers, next_round) cases: clean, broken link, bad signature, stale
    round, truncated signature, several peers, clock stop."""
    pk, bs = beacons()
    seed = bs[0].previous_sig
    out = [("clean", 0, seed, [bs], None), ("clock stop", 0, seed, [bs], 40), ("from mid-chain", 20, bs[19].signature, [bs[20:]], None)]
    bad = list(bs)
    bad[17] = Beacon(bad[17].previous_round, bad[17].previous_sig, bad[17].round, bs[18].signature)
    out.append(("bad signature then a second peer", 0, seed, [bad, bs[10:]], None))
    gap = list(bs)
    gap[30] = Beacon(gap[30].previous_round, bs[28].signature, gap[30].round, gap[30].signature)
    out.append(("broken prev sig", 0, seed, [gap], None))
    stale = bs[:12] + [bs[5]] + bs[12:]
    out.append(("stale round", 0, seed, [stale], None))
    short = list(bs)
    short[9] = Beacon(short[9].previous_round, short[9].previous_sig, short[9].round, short[9].signature[:48])
    out.append(("truncated signature", 0, seed, [short, bs[8:]], None))
    out.append(("empty peer then good", 0, seed, [[], bs[:33]], 30))
    out.append(("peer starts too late", 0, seed, [bs[3:], bs], None))
    return pk, out


@pytest.mark.parametrize("batch", [1, 3, 7, 64, 1000])
def test_sync_from_matches_reference_loop(batch):
    pk, cases = scenarios()
    for name, r0, s0, peers, nxt in cases:
        got_store = []
        res = bulk.sync_from(pk, r0, s0, peers, put=got_store.append, next_round=nxt, batch=batch, **CPU)
        want, err = ref_sync_from(pk, r0, s0, peers, nxt)
        assert got_store == want, name
        assert res.stored == len(want) and (res.error is None) == (err is None), name
        assert res.round == (want[-1].round if want else r0), name


def test_beacon_json_store_encoding():
    """json.Marshal of beacon.Beacon: declared field order, compact, []byte as std base64, and the
    BoltDB key roundToBytes."""
    b = Beacon(1, b"\x01\x02", 2, b"\xff" * 3)
    assert b.marshal() == b'{"PreviousRound":1,"PreviousSig":"AQI=","Round":2,"Signature":"////"}'
    assert Beacon.unmarshal(b.marshal()) == b
    assert Beacon.unmarshal(b'{"Round":7,"PreviousSig":null}') == Beacon(0, b"", 7, b"")
    for bad in (b"[]", b'{"Round":-1}', b'{"Round":"7"}', b'{"Signature":"***"}', b"{"):
        with pytest.raises(ValueError):
            Beacon.unmarshal(bad)
    assert bulk.round_to_bytes(258) == b"\x00\x00\x00\x00\x00\x00\x01\x02"
    _, bs = beacons()
    for x in bs[:4]:
        d = json.loads(x.marshal())
        assert base64.b64decode(d["Signature"]) == x.signature and d["Round"] == x.round


def store_records():
    pk, bs = beacons()
    recs = [(bulk.round_to_bytes(b.round), b.marshal()) for b in bs]
    want = np.zeros(len(recs), np.uint8)
    recs[5] = (recs[5][0], recs[5][1][:-3])                       # truncated JSON
    want[5] = bulk.ST_BAD_RECORD
    recs[9] = (bulk.round_to_bytes(99), recs[9][1])               # key != round
    want[9] = bulk.ST_BAD_RECORD
    b = bs[20]
    recs[20] = (recs[20][0], Beacon(b.previous_round, b.previous_sig, b.round, bs[21].signature).marshal())
    want[20] = 1                                                  # wrong signature ...
    want[21] = bulk.ST_BROKEN_LINK                                # ... so the next record's prev sig differs
    b = bs[40]
    recs[40] = (recs[40][0], Beacon(b.previous_round - 1, b.previous_sig, b.round, b.signature).marshal())
    want[40] = 1  # prev round is part of the message: the signature no longer verifies
    del recs[50]                                                  # a hole in the chain
    want = np.delete(want, 50)
    want[50] = bulk.ST_BROKEN_LINK
    return pk, bs, recs, want


def test_audit_chain_host_logic():
    pk, bs, recs, want = store_records()
    rep = bulk.audit_chain(pk, recs, batch=16, verify=twin_verify, randomness=twin_randomness)
    assert rep.status.tolist() == want.tolist()
    assert bytes(rep.randomness[0]) == bs[0].randomness()


def public_responses():
    pk, bs = beacons()
    rs = [PublicRand(b.previous_sig, b.previous_round, b.round, b.signature, b.randomness()) for b in bs[:16]]
    want = [0] * 16
    rs[2].randomness = None
    want[2] = bulk.ST_NO_RANDOMNESS
    rs[3].randomness = b""
    want[3] = bulk.ST_NO_RANDOMNESS
    rs[4].randomness = bs[5].randomness()
    want[4] = bulk.ST_BAD_RANDOMNESS
    rs[6].signature = bs[7].signature
    want[6] = 1
    rs[8].round += 1
    want[8] = 1
    rs[10].signature = b"\x00" * 96
    want[10] = 2
    return pk, rs, want


def test_verify_public_rand_host_logic():
    pk, rs, want = public_responses()
    assert bulk.verify_public_rand(pk, rs, verify=twin_verify, randomness=twin_randomness).tolist() == want


@pytest.mark.gpu
@pytest.mark.parametrize("batch", [3, 64, 16384])
def test_sync_from_gpu(batch):
    pk, cases = scenarios()
    for name, r0, s0, peers, nxt in cases:
        got = []
        res = bulk.sync_from(pk, r0, s0, peers, put=got.append, next_round=nxt, batch=batch)
        want, err = ref_sync_from(pk, r0, s0, peers, nxt)
        assert got == want and (res.error is None) == (err is None), name


@pytest.mark.gpu
def test_audit_chain_gpu():
    pk, bs, recs, want = store_records()
    rep = bulk.audit_chain(pk, recs)
    assert rep.status.tolist() == want.tolist()
    ok = rep.status == 0
    assert all(bytes(rep.randomness[i]) == hashlib.sha256(Beacon.unmarshal(recs[i][1]).signature).digest()
               for i in np.nonzero(ok)[0])


@pytest.mark.gpu
def test_verify_public_rand_gpu():
    pk, rs, want = public_responses()
    assert bulk.verify_public_rand(pk, rs).tolist() == want
