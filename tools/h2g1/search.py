"""Bounded search for the hash-to-G1 of the reference's test/test-integration/test.json (tooling, test data only).

json_output.go (kyber @ 20191229, signatures on G1) wrote Previous = x H1("Test Signature") and Public = x g2, so
e(Previous, g2) == e(H1("Test Signature"), Public) holds for the H1 that kyber's bls12-381 adapter used.  This script
tries a committed list of candidate H1 constructions (tools/h2g1/candidates.py) and compares the pairings through the
CPU twin (oracle/twin pairing_cubed: e^3, injective on the r-torsion).  Each candidate is tried with the six
automorphisms of E1 applied (+-P, (w x, +-y)): a map equal up to an automorphism is reported as such.

    python tools/h2g1/search.py            -> prints every hit (or "no hit") and writes tools/h2g1/result.json
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from oracle import twin  # noqa: E402
from oracle.pyref import bls12381 as B  # noqa: E402
from tools.h2g1 import candidates as C  # noqa: E402

P = B.P
W = None  # a primitive cube root of unity in Fp: (w x, y) is an automorphism of y^2 = x^3 + 4


def cube_root_of_unity():
    for g in range(2, 50):
        w = pow(g, (P - 1) // 3, P)
        if w != 1:
            return w
    raise RuntimeError


def g1_bytes(x, y):
    return B.g1_compress((B._FpWrap(x), B._FpWrap(y)))


def variants(pt):
    x, y = pt
    w = cube_root_of_unity()
    for xx in (x, x * w % P, x * w * w % P):
        for yy in (y, (-y) % P):
            yield (xx, yy)


def main():
    fx = json.load(open(os.path.join(ROOT, "tests", "golden", "reference_test_json_points.json")))
    pts = {p["name"]: bytes.fromhex(p["hex"]) for p in fx["points"]}
    g2 = B.g2_compress(B.G2_GEN)
    st, target = twin.pairing_cubed(pts["Previous"], g2)
    assert st == 0
    msg = b"Test Signature"
    hits, tried = [], 0
    t0 = time.time()
    for name, pt in C.candidates(msg):
        tried += 1
        if pt is None:
            continue
        for k, (x, y) in enumerate(variants(pt)):
            s, e = twin.pairing_cubed(g1_bytes(x, y), pts["Public"])
            if s == 0 and e == target:
                hits.append({"candidate": name, "automorphism": k})
                print("HIT", name, "automorphism", k, flush=True)
    res = {"tried": tried, "hits": hits, "seconds": round(time.time() - t0, 1),
           "check": "e(Previous, g2) == e(H1('Test Signature'), Public), via the twin's pairing (cubed)"}
    json.dump(res, open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "result.json"), "w"), indent=1)
    print("tried", tried, "candidates;", "hits:" if hits else "no hit", hits)


if __name__ == "__main__":
    main()
