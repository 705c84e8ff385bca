"""Generate g2_torsion.json: signatures of the committed chain with a torsion component added
(sigma + E, E of order 13, 23 or 13*23 in E'(Fp2), outside G2) plus uncleared hash outputs (on the
curve, outside G2).  Such encodings decode and lie on the curve, so only a G2 subgroup check rejects
them -- the case the batched subgroup check over the MSM window sums (drand_amd/csrc/msm.h) must catch.
Pure-Python pyref arithmetic (test infrastructure).  Usage: python tests/golden/make_torsion.py"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
from oracle.pyref import bls12381 as B  # noqa: E402

H2 = 0x5D543A95414E7F1091D50792876A202CD91DE4547085ABAA68A205B2E5A7DDFA628F1CB4D9E82EF21537E293A6691AE1616EC6E786F0C70CF1C38E31C7238E5


def torsion_point(order, tag):
    """A point of exactly `order` in E'(Fp2): [r lam / order] Q for an uncleared hash output Q, where
    lam = h2 / (13 * 23) is the exponent of the torsion part (its 13- and 23-parts are Z/13 x Z/13 and
    Z/23 x Z/23, so [h2 / 13] already kills every point)."""
    for i in range(16):
        q = B.hash_to_g2_uncleared(b"torsion %s %d" % (tag, i))
        e = B.G2C.mul(q, B.R * (H2 // (13 * 23) // order))
        if e is not None:
            assert B.G2C.mul(e, order) is None
            return e
    raise RuntimeError("no point of order %d" % order)


def main():
    chain = json.load(open(os.path.join(HERE, "chain_t3n5.json")))
    cases = []
    for order, rnd in ((13, 5), (23, 17), (13 * 23, 30), (13, 41)):
        e = torsion_point(order, b"%d" % order)
        sig = B.g2_decompress(bytes.fromhex(chain["rounds"][rnd]["sig"]))
        bad = B.G2C.add(sig, e)
        enc = B.g2_compress(bad)
        B.g2_decompress(enc, subgroup_check=False)  # decodes, on the curve
        assert not B.g2_in_subgroup(bad)
        cases.append({"round_index": rnd, "kind": "sigma + E, ord(E) = %d" % order, "sig": enc.hex()})
    for rnd in (9, 50):
        q = B.hash_to_g2_uncleared(bytes.fromhex(chain["rounds"][rnd]["msg"]))
        assert not B.g2_in_subgroup(q)
        cases.append({"round_index": rnd, "kind": "uncleared hash of the round's message", "sig": B.g2_compress(q).hex()})
    out = {"note": "chain_t3n5.json signatures replaced by on-curve points outside G2 (tests/golden/make_torsion.py)",
           "cases": cases}
    with open(os.path.join(HERE, "g2_torsion.json"), "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
