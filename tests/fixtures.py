"""Fixture loading and synthetic groups shared by the tests (tests/ only)."""
import json
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
GOLDEN = os.path.join(HERE, "golden")


def load(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


def hx(s):
    return bytes.fromhex(s)


def chain():
    """The committed 64-round C1 (n=5, t=3) chain."""
    return load("chain_t3n5.json")


def chain_arrays(c, rounds=None):
    rs = c["rounds"] if rounds is None else rounds
    pr = [r["prev_round"] for r in rs]
    rr = [r["round"] for r in rs]
    ps = [hx(r["prev_sig"]) for r in rs]
    sigs = np.frombuffer(b"".join(hx(r["sig"]) for r in rs), np.uint8).reshape(-1, 96).copy()
    msgs = np.frombuffer(b"".join(hx(r["msg"]) for r in rs), np.uint8).reshape(-1, 32).copy()
    return pr, rr, ps, sigs, msgs


def group(t, n):
    """Synthetic (t, n) group of tools/synthetic.py: commits via the CPU twin, shares as ints."""
    from oracle import twin
    from tools import synthetic as S

    coeffs = S.poly_coeffs(t)
    commits = [twin.g1_mul_gen(c) for c in coeffs]
    shares = [(i, S.share_value(coeffs, i)) for i in range(n)]
    return coeffs, commits, shares
