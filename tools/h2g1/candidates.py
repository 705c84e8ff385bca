"""Candidate hash-to-G1 constructions for the bounded test.json search (tools/h2g1/search.py).

The library that produced test.json (drand/kyber's bls12381 adapter over drand/bls12-381, go.mod:9-10 of the reference)
is absent from /root/reference, so these restate the constructions it could have used: the hash-to-curve draft's SSWU
map through the 11-isogeny (several DSTs, expand_message variants, sign conventions and cofactor multipliers), plus
try-and-increment and hash-to-scalar constructions.  The 11-isogeny is not typed in from memory: it is recomputed
here from E1' by factoring its 11-division polynomial and applying Velu's formulas, and its codomain is checked to be
E1 (j = 0) before it is used; the E1' constants are checked by the point count (#E1' = #E1).
"""
import hashlib
import hmac
import json
import os
import random

from sympy.ntheory.residue_ntheory import nthroot_mod
from sympy.polys.domains import ZZ
from sympy.polys import galoistools as gt

from oracle.pyref import bls12381 as B

P, R = B.P, B.R
X_BLS = -0xD201000000010000
N1 = P + 1 - (X_BLS + 1)                       # #E1(Fp)
H1 = 0x396C8C005555E1568C00AAAB0000AAAB         # full G1 cofactor = N1 / r
H1_EFF = 0xD201000000010001                     # 1 - x, the draft's effective cofactor
A_ISO = 0x144698A3B8E9433D693A02C96D4982B0EA985383EE66A8D8E8981AEFD881AC98936F8DA0E0F97F5CF428082D584C1D
B_ISO = 0x12E2908D11688030018B12E8753EEE3B2016C1F0F24F4070A0B9C14FCEF35EF55A23215A316CEAA5D1CC48E98E172BE0
Z_ISO = 11
HERE = os.path.dirname(os.path.abspath(__file__))


def inv(a):
    return pow(a % P, P - 2, P)


def sqrt(a):
    a %= P
    s = pow(a, (P + 1) // 4, P)
    return s if s * s % P == a else None


# ------------------------------------------------------------------ short Weierstrass arithmetic over Fp, affine
def add(c, p1, p2):
    a = c[0]
    if p1 is None:
        return p2
    if p2 is None:
        return p1
    (x1, y1), (x2, y2) = p1, p2
    if x1 == x2:
        if (y1 + y2) % P == 0:
            return None
        lam = (3 * x1 * x1 + a) * inv(2 * y1) % P
    else:
        lam = (y2 - y1) * inv(x2 - x1) % P
    x3 = (lam * lam - x1 - x2) % P
    return (x3, (lam * (x1 - x3) - y1) % P)


def mul(c, pt, k):
    acc = None
    while k:
        if k & 1:
            acc = add(c, acc, pt)
        pt = add(c, pt, pt)
        k >>= 1
    return acc


E1 = (0, 4)
E1P = (A_ISO, B_ISO)


def random_point(c, rng):
    while True:
        x = rng.randrange(P)
        y = sqrt(x * x * x + c[0] * x + c[1])
        if y is not None:
            return (x, y)


# ------------------------------------------------------------------ the 11-isogeny E1' -> E1, recomputed
def _division_poly_11(a, b):
    """f_n with psi_n = f_n (n odd), psi_n = 2y f_n (n even); lists high->low over GF(P) for sympy's galoistools."""
    dom = ZZ

    def m(*ps):
        r = [1]
        for q in ps:
            r = gt.gf_mul(r, q, P, dom)
        return r

    def s(u, v):
        return gt.gf_sub(u, v, P, dom)

    F = [4, 0, 4 * a % P, 4 * b % P]
    f = {0: [], 1: [1], 2: [1],
         3: [3, 0, 6 * a % P, 12 * b % P, (-a * a) % P],
         4: [2, 0, 10 * a % P, 40 * b % P, (-10 * a * a) % P, (-8 * a * b) % P, (-16 * b * b - 2 * a ** 3) % P]}
    F2 = m(F, F)

    def get(n):
        if n in f:
            return f[n]
        k = n // 2
        if n % 2:
            if k % 2 == 0:
                r = s(m(F2, get(k + 2), get(k), get(k), get(k)), m(get(k - 1), get(k + 1), get(k + 1), get(k + 1)))
            else:
                r = s(m(get(k + 2), get(k), get(k), get(k)), m(F2, get(k - 1), get(k + 1), get(k + 1), get(k + 1)))
        else:
            r = m(get(k), s(m(get(k + 2), get(k - 1), get(k - 1)), m(get(k - 2), get(k + 1), get(k + 1))))
        f[n] = gt.gf_strip(r)
        return f[n]

    return get(11)


class Fq5:
    """Fp[t]/(D) for the degree-5 kernel polynomial D (coefficient lists high->low); D need not be irreducible: the
    trace of multiplication is still the sum over D's roots, which is all Velu's formulas need."""

    def __init__(self, D):
        self.D = D

    def red(self, u):
        return gt.gf_rem(u, self.D, P, ZZ)

    def mul(self, u, v):
        return self.red(gt.gf_mul(u, v, P, ZZ))

    def inv(self, u):
        a, _, h = gt.gf_gcdex(u, self.D, P, ZZ)
        assert h == [1], "not invertible"
        return a

    def trace(self, u):
        tr = 0
        for j in range(5):
            w = self.mul(u, [1] + [0] * j)
            w = [0] * (5 - len(w)) + w
            tr += w[4 - j]
        return tr % P


def _velu(D, a, b):
    q = Fq5(D)
    t = [1, 0]
    t2 = q.mul(t, t)
    v = gt.gf_add_ground(gt.gf_mul_ground(t2, 6, P, ZZ), 2 * a % P, P, ZZ)
    u = gt.gf_mul_ground(gt.gf_add_ground(gt.gf_add(q.mul(t2, t), gt.gf_mul_ground(t, a, P, ZZ), P, ZZ), b, P, ZZ),
                         4, P, ZZ)
    A2 = (a - 5 * q.trace(v)) % P
    B2 = (b - 7 * q.trace(gt.gf_add(u, q.mul(t, v), P, ZZ))) % P
    return q, v, u, A2, B2


def isogeny():
    """Return (D, lam): kernel polynomial (high->low) and the isomorphism scale onto y^2 = x^3 + 4; cached."""
    cache = os.path.join(HERE, "iso11.json")
    if os.path.exists(cache):
        d = json.load(open(cache))
        return d["D"], d["lam"]
    rng = random.Random(1)
    pt = random_point(E1P, rng)
    assert mul(E1P, pt, N1) is None, "E1' constants: point count differs from E1"
    f11 = gt.gf_monic(_division_poly_11(A_ISO, B_ISO), P, ZZ)[1]
    found = None
    # the kernel's five x-coordinates form one Galois-stable set: either five rational roots (their product is the
    # degree-1 part of the distinct-degree factorisation) or one irreducible quintic
    kernels = []
    for g, deg in gt.gf_ddf_zassenhaus(f11, P, ZZ):
        if deg == 1 and len(g) - 1 == 5:
            kernels.append(g)
        elif deg == 5:
            kernels.extend(gt.gf_edf_zassenhaus(g, 5, P, ZZ))
    for D in kernels:
        if True:
            _, _, _, A2, B2 = _velu(D, A_ISO, B_ISO)
            if A2 == 0:
                c = 4 * inv(B2) % P
                lam = nthroot_mod(c, 6, P)
                if lam is not None:
                    found = (D, int(lam))
                    break
        if found:
            break
    assert found, "no 11-isogeny from E1' onto a curve isomorphic to E1 found"
    json.dump({"D": [int(x) for x in found[0]], "lam": found[1]}, open(cache, "w"))
    return found


_ISO = None


def iso_map(pt):
    global _ISO
    if _ISO is None:
        D, lam = isogeny()
        q, v, u, _, _ = _velu(D, A_ISO, B_ISO)
        _ISO = (q, v, u, lam)
    q, v, u, lam = _ISO
    if pt is None:
        return None
    x, y = pt
    d = gt.gf_sub_ground([1, 0], x, P, ZZ)            # t - x
    di = q.inv(d)                                     # 1/(t - x)
    di2 = q.mul(di, di)
    di3 = q.mul(di2, di)
    # X = x + sum v/(x - t) + u/(x - t)^2 ;  X' = 1 - sum v/(x - t)^2 + 2u/(x - t)^3 ; Y = y X'
    X = (x - q.trace(q.mul(v, di)) + q.trace(q.mul(u, di2))) % P
    Xd = (1 - q.trace(q.mul(v, di2)) + 2 * q.trace(q.mul(u, di3))) % P
    Y = y * Xd % P
    return (lam * lam * X % P, pow(lam, 3, P) * Y % P)


# ------------------------------------------------------------------ hash_to_field variants
def xmd(msg, dst, n, variant):
    H = hashlib.sha256
    if variant == "final":
        dstp = dst + bytes([len(dst)])
    else:                                             # early drafts: length prefix
        dstp = bytes([len(dst)]) + dst
    b0 = H(bytes(64) + msg + n.to_bytes(2, "big") + b"\x00" + dstp).digest()
    bi = H(b0 + b"\x01" + dstp).digest()
    out = bi
    for i in range(2, (n + 31) // 32 + 1):
        bi = H(bytes(x ^ y for x, y in zip(b0, bi)) + bytes([i]) + dstp).digest()
        out += bi
    return out[:n]


def hkdf_field(msg, dst, ctr, i=1):
    """draft-05 hash_to_base: HKDF-Extract(DST, msg || I2OSP(ctr, 1)), Expand(info = "H2C" || ctr || i, 64)."""
    prk = hmac.new(dst, msg + bytes([ctr]), hashlib.sha256).digest()
    info = b"H2C" + bytes([ctr]) + bytes([i])
    okm, t, k = b"", b"", 1
    while len(okm) < 64:
        t = hmac.new(prk, t + info + bytes([k]), hashlib.sha256).digest()
        okm += t
        k += 1
    return int.from_bytes(okm[:64], "big") % P


def fields(msg, dst, count, how):
    if how in ("final", "prefix"):
        ub = xmd(msg, dst, 64 * count, how)
        return [int.from_bytes(ub[64 * i:64 * i + 64], "big") % P for i in range(count)]
    return [hkdf_field(msg, dst, i) for i in range(count)]


# ------------------------------------------------------------------ SSWU onto E1'
def sgn0(v, how):
    v %= P
    return v & 1 if how == "parity" else int(v > (P - 1) // 2)


def sswu(u, how):
    A, Bc, Z = A_ISO, B_ISO, Z_ISO
    zu2 = Z * u * u % P
    den = (zu2 * zu2 + zu2) % P
    x1 = Bc * inv(Z * A) % P if den == 0 else (-Bc) * inv(A) * (1 + inv(den)) % P
    gx1 = (x1 ** 3 + A * x1 + Bc) % P
    y = sqrt(gx1)
    x = x1
    if y is None:
        x = zu2 * x1 % P
        y = sqrt(x ** 3 + A * x + Bc)
    if sgn0(u, how) != sgn0(y, how):
        y = (-y) % P
    return (x, y)


DSTS = [b"BLS_SIG_BLS12381G1_XMD:SHA-256_SSWU_RO_NUL_", b"BLS_SIG_BLS12381G1_XMD:SHA-256_SSWU_RO_POP_",
        b"BLS12381G1_XMD:SHA-256_SSWU_RO_", b"BLS12381G1_XMD:SHA-256_SSWU_NU_", b"BLS_SIG_BLS12381G1_XMD:SHA-256_SSWU_RO_",
        b"BLS_SIG_BLS12381G2_XMD:SHA-256_SSWU_RO_NUL_", b"QUUX-V01-CS02-with-BLS12381G1_XMD:SHA-256_SSWU_RO_", b""]


def sswu_candidates(msg):
    for dst in DSTS:
        for how in ("final", "prefix", "hkdf"):
            for count in (2, 1):
                us = fields(msg, dst, count, how)
                for sg in ("parity", "be"):
                    pts = [sswu(u, sg) for u in us]
                    for order in ("add_then_iso", "iso_then_add"):
                        if order == "add_then_iso":
                            q = None
                            for p_ in pts:
                                q = add(E1P, q, p_)
                            q = iso_map(q)
                        else:
                            q = None
                            for p_ in pts:
                                q = add(E1, q, iso_map(p_))
                        for cname, h in (("h_eff", H1_EFF), ("h", H1)):
                            yield (f"sswu dst={dst.decode()!r} field={how} count={count} sgn0={sg} {order} "
                                   f"cofactor={cname}", mul(E1, q, h))


def tai_candidates(msg):
    """try-and-increment: x = H(ctr || msg) or H(msg || ctr) mod p until x^3 + 4 is square, then clear cofactor."""
    for hname in ("sha256", "sha512", "blake2b"):
        for form in ("ctr_first", "ctr_last", "ctr_last_u32"):
            for ctr0 in (0, 1):
                pt = None
                for ctr in range(ctr0, ctr0 + 256):
                    cb = ctr.to_bytes(4, "big") if form == "ctr_last_u32" else bytes([ctr])
                    data = cb + msg if form == "ctr_first" else msg + cb
                    x = int.from_bytes(hashlib.new(hname, data).digest(), "big") % P
                    y = sqrt(x ** 3 + 4)
                    if y is not None:
                        pt = (x, y)
                        break
                for cname, h in (("h_eff", H1_EFF), ("h", H1)):
                    yield f"tai {hname} {form} start={ctr0} cofactor={cname}", (None if pt is None else mul(E1, pt, h))


def xinc_candidates(msg):
    """x0 = int(H(msg)) (or H of a domain-prefixed msg), then x += 1 until x^3 + 4 is square; clear cofactor."""
    for hname in ("sha256", "sha512", "blake2b", "sha3_256", "sha384"):
        for pre in (b"", b"BLS12381G1", b"BLS_SIG_BLS12381G1_XMD:SHA-256_SSWU_RO_NUL_"):
            x = int.from_bytes(hashlib.new(hname, pre + msg).digest(), "big") % P
            while sqrt(x ** 3 + 4) is None:
                x += 1
            pt = (x, sqrt(x ** 3 + 4))
            for cname, h in (("h_eff", H1_EFF), ("h", H1), ("none", 1)):
                yield f"x-increment {hname} prefix={pre!r} cofactor={cname}", mul(E1, pt, h)


def scalar_candidates(msg):
    g = (B.G1_GEN[0].v, B.G1_GEN[1].v)
    for hname in ("sha256", "sha512", "blake2b"):
        s = int.from_bytes(hashlib.new(hname, msg).digest(), "big") % R
        yield f"scalar {hname}(msg) * g1", mul(E1, g, s)


def candidates(msg):
    yield from scalar_candidates(msg)
    yield from xinc_candidates(msg)
    yield from tai_candidates(msg)
    yield from sswu_candidates(msg)
