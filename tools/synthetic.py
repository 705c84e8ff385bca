"""Deterministic synthetic drand group + chain definitions shared by tests, smoke() and bench.py.

Replaces kyber's `random.New()` (beacon/beacon_test.go:45, test/dkg.go) with a SHA-256 counter DRBG so
every run sees the same group and chain.  One master secret x signs the chain; the (n, t) groups of
BASELINE.json's configs are degree-(t-1) polynomials with p(0) = x, so every config's recovered
signature for round r equals the chain's sigma_r.

This module holds no curve arithmetic: commits / signatures are produced by whoever calls it
(the CPU twin for fixtures, the GPU for bulk partials).
"""
import hashlib

R = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001
# GenesisSeed of the reference's deploy/200409/group.toml:5 used as round-0 "signature".
GENESIS_SEED = bytes.fromhex("770f3c2578a95387b358e02aba5d5008a53ce40047a1fa326dde0dfd0b482a8e")
LABEL = b"drand-amd/synthetic/v1"


def drbg_scalar(label, counter):
    h = hashlib.sha256(LABEL + b"/" + label + b"/" + counter.to_bytes(8, "big")).digest()
    h2 = hashlib.sha256(h + b"/2").digest()
    return int.from_bytes(h + h2, "big") % R


def master_secret():
    return drbg_scalar(b"master", 0)


def poly_coeffs(t):
    """Coefficients a_0..a_{t-1} with a_0 = the master secret."""
    return [master_secret()] + [drbg_scalar(b"poly-t%d" % t, j) for j in range(1, t)]


def share_value(coeffs, i):
    """PriPoly share of index i (x = i + 1), kyber share.PriPoly.Eval."""
    x = i + 1
    acc = 0
    for c in reversed(coeffs):
        acc = (acc * x + c) % R
    return acc


def chain_path(n):
    import os
    return os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "data", "chain_v1_%d.bin" % n)


# SHA-256 of the chain files tools/gen_chain.py wrote with the CPU twin (data/ is git-ignored; the files travel to
# the GPU box with the tree).  A chain file is trusted only if it matches: the GPU library under test must never
# have produced the rounds it verifies.
CHAIN_SHA256 = {
    100000: "bd4426dc5132c730295720ec0ba6ecc5ef44d5c500e2c4c581d550cd49a3e9f0",
    1000000: "5b33b619c02f415f794497b4cc84abcc1144e73d6bb4a35787366fa126d627a4",
}


class ChainFileError(RuntimeError):
    pass


def chain_file_sha256(path):
    h = hashlib.sha256()
    with open(path, "rb") as f:
        for blk in iter(lambda: f.read(1 << 22), b""):
            h.update(blk)
    return h.hexdigest()


def find_chain(total, data_dir=None):
    """(n, path) of the smallest digest-pinned chain file data/chain_v1_<n>.bin with n >= total.  Raises
    ChainFileError when none covers `total` or when the covering file does not match its pinned SHA-256."""
    import os

    d = data_dir or os.path.dirname(chain_path(1))
    have = sorted(n for n in CHAIN_SHA256 if n >= total and os.path.exists(os.path.join(d, "chain_v1_%d.bin" % n)))
    if not have:
        raise ChainFileError("no chain file covers %d rounds in %s (pinned sizes: %s; tools/gen_chain.py makes them)"
                             % (total, d, sorted(CHAIN_SHA256)))
    n = have[0]
    p = os.path.join(d, "chain_v1_%d.bin" % n)
    got = chain_file_sha256(p)
    if got != CHAIN_SHA256[n]:
        raise ChainFileError("%s: SHA-256 %s does not match the pinned %s" % (p, got, CHAIN_SHA256[n]))
    return n, p


# x * g1 for x = master_secret(): the group key C_0 of every synthetic group (= chain_t3n5.json "pk";
# pinned by tests/test_oracle.py::test_group_pk_constant)
GROUP_PK = bytes.fromhex("a48a078a2548dcc710aa9925a1c0cf951be802bdce52febb5f1b75af1a01c22760724cd295bdc4fe7e5ab0f6cead0564")
