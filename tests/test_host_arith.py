"""The kernels' device arithmetic compiled for the host (tests/native/hostcheck.cpp, g++): the same
field/curve/hash code that runs on gfx950, checked on CPU against the oracle and the fixtures."""
import ctypes
import os
import random
import subprocess

import pytest

from oracle.pyref import bls12381 as B
from tests.fixtures import hx, load

HERE = os.path.dirname(os.path.abspath(__file__))
NATIVE = os.path.join(HERE, "native")


@pytest.fixture(scope="module")
def hc():
    subprocess.run(["make", "-s", "-C", NATIVE], check=True)
    return ctypes.CDLL(os.path.join(NATIVE, "libhostcheck.so"))


def test_fp_inv_safegcd_matches_fermat_and_python(hc):
    rng = random.Random(7)
    vals = [0, 1, 2, B.P - 1, B.P - 2, (1 << 380) + 12345] + [rng.randrange(B.P) for _ in range(300)]
    for a in vals:
        sg = ctypes.create_string_buffer(48)
        fe = ctypes.create_string_buffer(48)
        hc.hc_fp_inv(a.to_bytes(48, "big"), sg, fe)
        want = pow(a, B.P - 2, B.P)
        assert int.from_bytes(sg.raw, "big") == want, hex(a)
        assert fe.raw == sg.raw


def test_hash_to_g2_host_build_matches_golden(hc):
    v = load("hash_to_g2_nul.json")
    dst = v["dst"].encode()
    for x in v["vectors"][:4]:
        out = ctypes.create_string_buffer(96)
        m = hx(x["msg"])
        hc.hc_hash_to_g2(m, len(m), dst, len(dst), out)
        assert out.raw.hex() == x["h"]
