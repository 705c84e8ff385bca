"""Pure-Python BLS12-381 restatement -- TEST INFRASTRUCTURE ONLY (the oracle).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this.
It is the independent checker for the HIP path, never the thing measured or shipped.

What it restates (the reference's arithmetic lives in un-vendored modules):
  * github.com/drand/bls12-381 @ v0.2.0 (go.mod:9)      -- field tower, curves, ZCash compression,
    hash-to-G2, optimal-ate pairing.  Restated from the published BLS12-381 / RFC 9380 algorithms.
  * the suite is selected in key/curve.go:12 (`bls.NewBLS12381Suite()`), keys on G1 (key/curve.go:21),
    signatures on G2 (key/curve.go:26).

Representation choices are deliberately different from the HIP kernels so the two are independent:
python ints, affine points with field inversions, and the pairing computed on the *untwisted* curve
over Fp12 = Fp[w]/(w^12 - 2 w^6 + 2) (no tower, no sparse lines, plain final exponentiation).

Parity pinning (see tests/test_oracle_kat.py): generator encodings, RFC 9380 expand_message_xmd and
hash_to_curve(G2) known-answer vectors, and the G1 keys held by the reference in
deploy/200409/group.toml and demo/docker/data/group.toml.
"""
import hashlib

P = 0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFAAAB
R = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001
Z_ABS = 0xD201000000010000  # BLS parameter z = -Z_ABS

# Domain separation tag of the hash-to-G2 variant (single switch).
DST_G2 = b"BLS_SIG_BLS12381G2_XMD:SHA-256_SSWU_RO_NUL_"


def inv(a):
    return pow(a, P - 2, P)


def legendre(a):
    a %= P
    if a == 0:
        return 0
    return 1 if pow(a, (P - 1) // 2, P) == 1 else -1


def fp_sqrt(a):
    a %= P
    s = pow(a, (P + 1) // 4, P)
    return s if s * s % P == a else None


# ----------------------------------------------------------------------------- Fp2 = Fp[u]/(u^2+1)
class Fp2:
    __slots__ = ("c0", "c1")

    def __init__(self, c0, c1=0):
        self.c0 = c0 % P
        self.c1 = c1 % P

    def __add__(s, o):
        return Fp2(s.c0 + o.c0, s.c1 + o.c1)

    def __sub__(s, o):
        return Fp2(s.c0 - o.c0, s.c1 - o.c1)

    def __neg__(s):
        return Fp2(-s.c0, -s.c1)

    def __mul__(s, o):
        if isinstance(o, int):
            return Fp2(s.c0 * o, s.c1 * o)
        return Fp2(s.c0 * o.c0 - s.c1 * o.c1, s.c0 * o.c1 + s.c1 * o.c0)

    __rmul__ = __mul__

    def __eq__(s, o):
        return s.c0 == o.c0 and s.c1 == o.c1

    def __hash__(s):
        return hash((s.c0, s.c1))

    def __repr__(s):
        return "Fp2(%#x, %#x)" % (s.c0, s.c1)

    def is_zero(s):
        return s.c0 == 0 and s.c1 == 0

    def conj(s):
        return Fp2(s.c0, -s.c1)

    def norm(s):
        return (s.c0 * s.c0 + s.c1 * s.c1) % P

    def inv(s):
        n = inv(s.norm())
        return Fp2(s.c0 * n, -s.c1 * n)

    def __pow__(s, e):
        r = Fp2(1)
        b = s
        while e:
            if e & 1:
                r = r * b
            b = b * b
            e >>= 1
        return r

    def is_square(s):
        return legendre(s.norm()) != -1

    def sqrt(s):
        """Any square root, or None.  Adj & Rodriguez-Henriquez, Alg. 9 (p = 3 mod 4)."""
        if s.is_zero():
            return Fp2(0)
        a1 = s ** ((P - 3) // 4)
        alpha = a1 * a1 * s
        a0 = (alpha ** P) * alpha
        if a0 == Fp2(-1):
            return None
        x0 = a1 * s
        if alpha == Fp2(-1):
            x = Fp2(0, 1) * x0
        else:
            b = (Fp2(1) + alpha) ** ((P - 1) // 2)
            x = b * x0
        return x if x * x == s else None


def sgn0_fp2(a):
    """RFC 9380 §4.1 sgn0 for m = 2."""
    sign_0 = a.c0 & 1
    zero_0 = a.c0 == 0
    sign_1 = a.c1 & 1
    return sign_0 | (zero_0 & sign_1)


def fp_lex_largest(y):
    return y > (P - 1) // 2


def fp2_lex_largest(y):
    """ZCash serialization 'sort' flag for Fp2: compare c1 first, then c0."""
    if y.c1 != 0:
        return y.c1 > (P - 1) // 2
    return y.c0 > (P - 1) // 2


# ----------------------------------------------------------------------------- generic affine curve
# Points are (x, y) tuples of field elements, None is the point at infinity.
class Curve:
    def __init__(self, b, zero, one):
        self.b = b
        self.zero = zero
        self.one = one

    def on_curve(self, pt):
        if pt is None:
            return True
        x, y = pt
        return y * y == x * x * x + self.b

    def neg(self, pt):
        if pt is None:
            return None
        return (pt[0], -pt[1])

    def _inv(self, a):
        return a.inv() if not isinstance(a, int) else inv(a)

    def add(self, p1, p2):
        if p1 is None:
            return p2
        if p2 is None:
            return p1
        x1, y1 = p1
        x2, y2 = p2
        if x1 == x2:
            if y1 == y2:
                return self.double(p1)
            return None
        lam = (y2 - y1) * self._inv(x2 - x1)
        x3 = lam * lam - x1 - x2
        return (x3, lam * (x1 - x3) - y1)

    def double(self, p1):
        if p1 is None:
            return None
        x, y = p1
        if y == self.zero:
            return None
        lam = (x * x * 3) * self._inv(y * 2)
        x3 = lam * lam - x * 2
        return (x3, lam * (x - x3) - y)

    def mul(self, pt, k):
        if k < 0:
            return self.mul(self.neg(pt), -k)
        acc = None
        add = pt
        while k:
            if k & 1:
                acc = self.add(acc, add)
            add = self.double(add)
            k >>= 1
        return acc

    def eq(self, p1, p2):
        if p1 is None or p2 is None:
            return p1 is None and p2 is None
        return p1[0] == p2[0] and p1[1] == p2[1]


class _FpWrap:
    """Minimal Fp element with operator overloads so Curve works over Fp."""
    __slots__ = ("v",)

    def __init__(self, v):
        self.v = v % P

    def __add__(s, o):
        return _FpWrap(s.v + o.v)

    def __sub__(s, o):
        return _FpWrap(s.v - o.v)

    def __neg__(s):
        return _FpWrap(-s.v)

    def __mul__(s, o):
        if isinstance(o, int):
            return _FpWrap(s.v * o)
        return _FpWrap(s.v * o.v)

    __rmul__ = __mul__

    def __eq__(s, o):
        return s.v == o.v

    def inv(s):
        return _FpWrap(inv(s.v))


G1C = Curve(_FpWrap(4), _FpWrap(0), _FpWrap(1))
XI = Fp2(1, 1)
G2C = Curve(Fp2(4, 4), Fp2(0), Fp2(1))

G1_GEN = (
    _FpWrap(0x17F1D3A73197D7942695638C4FA9AC0FC3688C4F9774B905A14E3A3F171BAC586C55E83FF97A1AEFFB3AF00ADB22C6BB),
    _FpWrap(0x08B3F481E3AAA0F1A09E30ED741D8AE4FCF5E095D5D00AF600DB18CB2C04B3EDD03CC744A2888AE40CAA232946C5E7E1),
)
G2_GEN = (
    Fp2(
        0x024AA2B2F08F0A91260805272DC51051C6E47AD4FA403B02B4510B647AE3D1770BAC0326A805BBEFD48056C8C121BDB8,
        0x13E02B6052719F607DACD3A088274F65596BD0D09920B61AB5DA61BBDC7F5049334CF11213945D57E5AC7D055D042B7E,
    ),
    Fp2(
        0x0CE5D527727D6E118CC9CDC6DA2E351AADFD9BAA8CBDD3A76D429A695160D12C923AC9CC3BACA289E193548608B82801,
        0x0606C4A02EA734CC32ACD2B02BC28B99CB3E287E85A763AF267492AB572E99AB3F370D275CEC1DA1AAA9075FF05F79BE,
    ),
)


# ----------------------------------------------------------------------------- ZCash encodings
class DecodeError(Exception):
    pass


def g1_compress(pt):
    if pt is None:
        return bytes([0xC0]) + bytes(47)
    x, y = pt
    b = bytearray(x.v.to_bytes(48, "big"))
    b[0] |= 0x80
    if fp_lex_largest(y.v):
        b[0] |= 0x20
    return bytes(b)


def g1_decompress(data, subgroup_check=True):
    """48 B ZCash G1 -> affine point (None = infinity); raises DecodeError."""
    if len(data) != 48:
        raise DecodeError("g1: bad length")
    f = data[0]
    if not f & 0x80:
        raise DecodeError("g1: compression flag not set")
    if f & 0x40:
        if f != 0xC0 or any(data[1:]):
            raise DecodeError("g1: bad infinity encoding")
        return None
    x = int.from_bytes(bytes([f & 0x1F]) + data[1:], "big")
    if x >= P:
        raise DecodeError("g1: x not canonical")
    y = fp_sqrt(x * x * x + 4)
    if y is None:
        raise DecodeError("g1: not on curve")
    if bool(f & 0x20) != fp_lex_largest(y):
        y = P - y
    pt = (_FpWrap(x), _FpWrap(y))
    if subgroup_check and G1C.mul(pt, R) is not None:
        raise DecodeError("g1: not in subgroup")
    return pt


def g2_compress(pt):
    if pt is None:
        return bytes([0xC0]) + bytes(95)
    x, y = pt
    b = bytearray(x.c1.to_bytes(48, "big") + x.c0.to_bytes(48, "big"))
    b[0] |= 0x80
    if fp2_lex_largest(y):
        b[0] |= 0x20
    return bytes(b)


def g2_decompress(data, subgroup_check=True):
    """96 B ZCash G2 (x = c1 || c0) -> affine point (None = infinity); raises DecodeError."""
    if len(data) != 96:
        raise DecodeError("g2: bad length")
    f = data[0]
    if not f & 0x80:
        raise DecodeError("g2: compression flag not set")
    if f & 0x40:
        if f != 0xC0 or any(data[1:]):
            raise DecodeError("g2: bad infinity encoding")
        return None
    x1 = int.from_bytes(bytes([f & 0x1F]) + data[1:48], "big")
    x0 = int.from_bytes(data[48:], "big")
    if x1 >= P or x0 >= P:
        raise DecodeError("g2: x not canonical")
    x = Fp2(x0, x1)
    y = (x * x * x + G2C.b).sqrt()
    if y is None:
        raise DecodeError("g2: not on curve")
    if bool(f & 0x20) != fp2_lex_largest(y):
        y = -y
    pt = (x, y)
    if subgroup_check and not g2_in_subgroup(pt):
        raise DecodeError("g2: not in subgroup")
    return pt


def g2_in_subgroup(pt):
    return G2C.mul(pt, R) is None


# ----------------------------------------------------------------------------- RFC 9380 hash_to_curve (G2)
def expand_message_xmd(msg, dst, len_in_bytes):
    """RFC 9380 §5.3.1 with H = SHA-256 (b_in_bytes = 32, s_in_bytes = 64)."""
    if len(dst) > 255:
        dst = hashlib.sha256(b"H2C-OVERSIZE-DST-" + dst).digest()
    ell = (len_in_bytes + 31) // 32
    assert ell <= 255
    dst_prime = dst + bytes([len(dst)])
    z_pad = bytes(64)
    l_i_b = len_in_bytes.to_bytes(2, "big")
    b0 = hashlib.sha256(z_pad + msg + l_i_b + b"\x00" + dst_prime).digest()
    bi = hashlib.sha256(b0 + b"\x01" + dst_prime).digest()
    out = bi
    for i in range(2, ell + 1):
        bi = hashlib.sha256(bytes(a ^ b for a, b in zip(b0, bi)) + bytes([i]) + dst_prime).digest()
        out += bi
    return out[:len_in_bytes]


def hash_to_field_fp2(msg, count, dst):
    L = 64
    ub = expand_message_xmd(msg, dst, count * 2 * L)
    out = []
    for i in range(count):
        e = []
        for j in range(2):
            off = L * (j + i * 2)
            e.append(int.from_bytes(ub[off : off + L], "big") % P)
        out.append(Fp2(e[0], e[1]))
    return out


# 3-isogenous curve E2': y^2 = x^3 + A' x + B'
SSWU_A = Fp2(0, 240)
SSWU_B = Fp2(1012, 1012)
SSWU_Z = Fp2(-2, -1)


def map_to_curve_sswu(u):
    """RFC 9380 §6.6.2 simplified SWU onto E2' (straight-line restatement)."""
    A, B, Z = SSWU_A, SSWU_B, SSWU_Z
    zu2 = Z * u * u
    den = zu2 * zu2 + zu2
    if den.is_zero():
        x1 = B * (Z * A).inv()
    else:
        x1 = (-B) * A.inv() * (Fp2(1) + den.inv())
    gx1 = x1 * x1 * x1 + A * x1 + B
    if gx1.is_square():
        x, y = x1, gx1.sqrt()
    else:
        x2 = zu2 * x1
        gx2 = x2 * x2 * x2 + A * x2 + B
        x, y = x2, gx2.sqrt()
    if sgn0_fp2(u) != sgn0_fp2(y):
        y = -y
    return (x, y)


def _h(s):
    return int(s, 16)


# RFC 9380 Appendix E.3 3-isogeny constants (validated in tests against Velu's formulas and the
# RFC known-answer vector, see tests/test_oracle_kat.py).
ISO_XNUM = [
    Fp2(_h("5c759507e8e333ebb5b7a9a47d7ed8532c52d39fd3a042a88b58423c50ae15d5c2638e343d9c71c6238aaaaaaaa97d6"),
        _h("5c759507e8e333ebb5b7a9a47d7ed8532c52d39fd3a042a88b58423c50ae15d5c2638e343d9c71c6238aaaaaaaa97d6")),
    Fp2(0, _h("11560bf17baa99bc32126fced787c88f984f87adf7ae0c7f9a208c6b4f20a4181472aaa9cb8d555526a9ffffffffc71a")),
    Fp2(_h("11560bf17baa99bc32126fced787c88f984f87adf7ae0c7f9a208c6b4f20a4181472aaa9cb8d555526a9ffffffffc71e"),
        _h("8ab05f8bdd54cde190937e76bc3e447cc27c3d6fbd7063fcd104635a790520c0a395554e5c6aaaa9354ffffffffe38d")),
    Fp2(_h("171d6541fa38ccfaed6dea691f5fb614cb14b4e7f4e810aa22d6108f142b85757098e38d0f671c7188e2aaaaaaaa5ed1"), 0),
]
ISO_XDEN = [Fp2(0, -72), Fp2(12, -12), Fp2(1, 0)]
ISO_YNUM = [
    Fp2(_h("1530477c7ab4113b59a4c18b076d11930f7da5d4a07f649bf54439d87d27e500fc8c25ebf8c92f6812cfc71c71c6d706"),
        _h("1530477c7ab4113b59a4c18b076d11930f7da5d4a07f649bf54439d87d27e500fc8c25ebf8c92f6812cfc71c71c6d706")),
    Fp2(0, _h("5c759507e8e333ebb5b7a9a47d7ed8532c52d39fd3a042a88b58423c50ae15d5c2638e343d9c71c6238aaaaaaaa97be")),
    Fp2(_h("11560bf17baa99bc32126fced787c88f984f87adf7ae0c7f9a208c6b4f20a4181472aaa9cb8d555526a9ffffffffc71c"),
        _h("8ab05f8bdd54cde190937e76bc3e447cc27c3d6fbd7063fcd104635a790520c0a395554e5c6aaaa9354ffffffffe38f")),
    Fp2(_h("124c9ad43b6cf79bfbf7043de3811ad0761b0f37a1e26286b0e977c69aa274524e79097a56dc4bd9e1b371c71c718b10"), 0),
]
ISO_YDEN = [Fp2(-432, -432), Fp2(0, -216), Fp2(18, -18), Fp2(1, 0)]


def _poly(coeffs, x):
    acc = Fp2(0)
    for c in reversed(coeffs):
        acc = acc * x + c
    return acc


def iso_map(pt):
    if pt is None:
        return None
    x, y = pt
    xd = _poly(ISO_XDEN, x)
    yd = _poly(ISO_YDEN, x)
    if xd.is_zero() or yd.is_zero():
        return None
    return (_poly(ISO_XNUM, x) * xd.inv(), y * _poly(ISO_YNUM, x) * yd.inv())


# psi endomorphism (untwist-Frobenius-twist) on E2
PSI_CX = (XI ** ((P - 1) // 3)).inv()
PSI_CY = (XI ** ((P - 1) // 2)).inv()


def psi(pt):
    if pt is None:
        return None
    x, y = pt
    return (x.conj() * PSI_CX, y.conj() * PSI_CY)


H_EFF_G2 = _h(
    "bc69f08f2ee75b3584c6a0ea91b352888e2a8e9145ad7689986ff031508ffe1329c2f178731db956d82bf015d1212b02ec0ec69d7477c1ae954cbc06689f6a359894c0adebbf6b4e8020005aaa95551"
)


def clear_cofactor_g2(pt):
    """RFC 9380 §8.8.2: multiply by h_eff (computed here as a plain scalar multiplication)."""
    return G2C.mul(pt, H_EFF_G2)


def hash_to_g2(msg, dst=DST_G2):
    u0, u1 = hash_to_field_fp2(msg, 2, dst)
    q0 = iso_map(map_to_curve_sswu(u0))
    q1 = iso_map(map_to_curve_sswu(u1))
    return clear_cofactor_g2(G2C.add(q0, q1))


def hash_to_g2_uncleared(msg, dst=DST_G2):
    u0, u1 = hash_to_field_fp2(msg, 2, dst)
    return G2C.add(iso_map(map_to_curve_sswu(u0)), iso_map(map_to_curve_sswu(u1)))


# ----------------------------------------------------------------------------- pairing over Fp12 (untwisted)
# Fp12 = Fp[w]/(w^12 - 2 w^6 + 2); u = w^6 - 1 embeds Fp2, xi = 1+u = w^6.
class Fp12:
    __slots__ = ("c",)

    def __init__(self, c):
        self.c = [x % P for x in c]

    @staticmethod
    def one():
        return Fp12([1] + [0] * 11)

    def __add__(s, o):
        return Fp12([a + b for a, b in zip(s.c, o.c)])

    def __sub__(s, o):
        return Fp12([a - b for a, b in zip(s.c, o.c)])

    def __neg__(s):
        return Fp12([-a for a in s.c])

    def __mul__(s, o):
        if isinstance(o, int):
            return Fp12([a * o for a in s.c])
        prod = [0] * 23
        for i, a in enumerate(s.c):
            if a:
                for j, b in enumerate(o.c):
                    prod[i + j] += a * b
        # reduce with w^12 = 2 w^6 - 2
        for k in range(22, 11, -1):
            t = prod[k]
            if t:
                prod[k - 6] += 2 * t
                prod[k - 12] -= 2 * t
        return Fp12(prod[:12])

    __rmul__ = __mul__

    def __eq__(s, o):
        return s.c == o.c

    def is_one(s):
        return s.c[0] == 1 and not any(s.c[1:])

    def __pow__(s, e):
        r = Fp12.one()
        b = s
        while e:
            if e & 1:
                r = r * b
            b = b * b
            e >>= 1
        return r

    def inv(s):
        # Extended Euclid over Fp[w] against the modulus polynomial.
        mod = [2, 0, 0, 0, 0, 0, -2, 0, 0, 0, 0, 0, 1]
        lm, hm = [1] + [0] * 12, [0] * 13
        low, high = s.c + [0], [m % P for m in mod]

        def deg(p):
            d = len(p) - 1
            while d and p[d] % P == 0:
                d -= 1
            return d

        while deg(low):
            r = _poly_div(high, low)
            r += [0] * (13 - len(r))
            nm, new = hm[:], high[:]
            for i in range(13):
                for j in range(13 - i):
                    nm[i + j] -= lm[i] * r[j]
                    new[i + j] -= low[i] * r[j]
            nm = [x % P for x in nm]
            new = [x % P for x in new]
            lm, low, hm, high = nm, new, lm, low
        c = inv(low[0])
        return Fp12([x * c for x in lm[:12]])


def _poly_div(a, b):
    def deg(p):
        d = len(p) - 1
        while d and p[d] % P == 0:
            d -= 1
        return d

    dega, degb = deg(a), deg(b)
    temp = [x for x in a]
    o = [0] * len(a)
    ib = inv(b[degb])
    for i in range(dega - degb, -1, -1):
        o[i] = (o[i] + temp[degb + i] * ib) % P
        for c in range(degb + 1):
            temp[c + i] = (temp[c + i] - o[i] * b[c]) % P
    return [x % P for x in o[: deg(o) + 1]]


def _fp2_to_fp12(a):
    c = [0] * 12
    c[0] = a.c0 - a.c1
    c[6] = a.c1
    return Fp12(c)


_W = Fp12([0, 1] + [0] * 10)
_W2_INV = (_W * _W).inv()
_W3_INV = (_W * _W * _W).inv()
E12 = Curve(Fp12([4] + [0] * 11), Fp12([0] * 12), Fp12.one())


def untwist(q):
    """E2 -> E(Fp12): (x, y) -> (x / w^2, y / w^3) (M-type sextic twist)."""
    if q is None:
        return None
    return (_fp2_to_fp12(q[0]) * _W2_INV, _fp2_to_fp12(q[1]) * _W3_INV)


def _line(p1, p2, t):
    """Value at t of the line through p1, p2 (tangent if equal); vertical parts dropped."""
    x1, y1 = p1
    x2, y2 = p2
    xt, yt = t
    if x1 != x2:
        lam = (y2 - y1) * (x2 - x1).inv()
    elif y1 == y2:
        lam = x1 * x1 * 3 * (y1 * 2).inv()
    else:
        return xt - x1
    return lam * (xt - x1) - (yt - y1)


def miller_loop(q2, p1):
    """f_{z,Q}(P) on the untwisted curve, z = -Z_ABS (the 1/f is taken for the negative z)."""
    if q2 is None or p1 is None:
        return Fp12.one()
    Q = untwist(q2)
    Pt = (Fp12([p1[0].v] + [0] * 11), Fp12([p1[1].v] + [0] * 11))
    T = Q
    f = Fp12.one()
    for bit in bin(Z_ABS)[3:]:
        f = f * f * _line(T, T, Pt)
        T = E12.double(T)
        if bit == "1":
            f = f * _line(T, Q, Pt)
            T = E12.add(T, Q)
    return f.inv()


FINAL_EXP = (P ** 12 - 1) // R


def pairing(p1, q2):
    return miller_loop(q2, p1) ** FINAL_EXP


def pairing_check(pairs):
    """prod e(P_i, Q_i) == 1 with one shared final exponentiation."""
    f = Fp12.one()
    for p1, q2 in pairs:
        f = f * miller_loop(q2, p1)
    return (f ** FINAL_EXP).is_one()
