"""Commitments (48 B compressed G1, kyber PubPoly) of the synthetic (t, n) groups of tools/synthetic.py,
computed by the CPU twin and cross-checked with the pure-Python oracle; written to tests/golden/groups.json.
bench.py reads them (the GPU never needs a G1 scalar multiplication by a secret)."""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from oracle import twin  # noqa: E402
from oracle.pyref import bls12381 as B  # noqa: E402
from tools import synthetic as S  # noqa: E402


def main():
    out = {}
    for t in (3, 33, 129):
        coeffs = S.poly_coeffs(t)
        commits = [twin.g1_mul_gen(c) for c in coeffs]
        assert B.g1_compress(B.G1C.mul(B.G1_GEN, coeffs[-1])) == commits[-1]
        out["t%d" % t] = [c.hex() for c in commits]
    with open(os.path.join(HERE, "groups.json"), "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
    print("wrote groups.json")


if __name__ == "__main__":
    main()
