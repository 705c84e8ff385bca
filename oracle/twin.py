"""ctypes binding of the CPU twin (oracle/twin/twin.c) -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module.
"""
import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "twin", "libdrandtwin.so")
_lib = None

DST_NUL = b"BLS_SIG_BLS12381G2_XMD:SHA-256_SSWU_RO_NUL_"


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            raise RuntimeError("CPU twin not built: run `make -C oracle` (or __graft_entry__.build())")
        L = ctypes.CDLL(_LIB_PATH)
        c = ctypes
        P = c.c_void_p
        L.twin_init.restype = None
        L.twin_hash_to_g2.argtypes = [P, c.c_size_t, P, c.c_size_t, P]
        L.twin_sign.argtypes = [P, P, c.c_size_t, P]
        L.twin_verify.argtypes = [P, P, c.c_size_t, P]
        L.twin_verify_batch.argtypes = [P, c.c_size_t, P, c.c_size_t, P, P, c.c_int]
        L.twin_beacon_message.argtypes = [P, c.c_size_t, c.c_uint64, c.c_uint64, P]
        L.twin_gen_chain.argtypes = [P, P, c.c_size_t, c.c_uint64, c.c_size_t, P]
        L.twin_pubpoly_eval.argtypes = [P, c.c_uint32, c.c_uint32, P]
        L.twin_g1_mul_gen.argtypes = [P, P]
        L.twin_verify_partial.argtypes = [P, c.c_uint32, P, c.c_size_t, P, c.c_size_t]
        L.twin_recover.argtypes = [P, c.c_uint32, c.c_uint32, P, c.c_size_t, P, c.c_uint32, P, P]
        L.twin_recover_batch.argtypes = [P, c.c_uint32, c.c_uint32, c.c_size_t, P, P, c.c_uint32, P, P, P, c.c_int]
        L.twin_pairing_cubed.argtypes = [P, P, P]
        L.twin_set_dst.argtypes = [P, c.c_size_t]
        L.twin_c1_batch.argtypes = [P, c.c_uint32, c.c_uint32, P, c.c_size_t, P, P, c.c_int]
        L.twin_c1_batch.restype = c.c_size_t
        L.twin_opcount.restype = c.c_uint64
        L.twin_opcount_enable.argtypes = [c.c_int]
        L.twin_init()
        _lib = L
    return _lib


def _buf(b):
    return ctypes.c_char_p(bytes(b))


def _np_ptr(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def hash_to_g2(msg, dst=DST_NUL):
    out = ctypes.create_string_buffer(96)
    lib().twin_hash_to_g2(_buf(msg), len(msg), _buf(dst), len(dst), out)
    return out.raw


def sign(sk, msg):
    out = ctypes.create_string_buffer(96)
    lib().twin_sign(_buf(int(sk).to_bytes(32, "big")), _buf(msg), len(msg), out)
    return out.raw


def verify(pk48, msg, sig96):
    return lib().twin_verify(_buf(pk48), _buf(msg), len(msg), _buf(sig96))


def verify_batch(pk48, msgs, sigs, threads=1):
    """msgs: (n, L) uint8, sigs: (n, 96) uint8 -> status (n,) uint8."""
    msgs = np.ascontiguousarray(msgs, dtype=np.uint8)
    sigs = np.ascontiguousarray(sigs, dtype=np.uint8)
    n = sigs.shape[0]
    st = np.zeros(n, dtype=np.uint8)
    lib().twin_verify_batch(_buf(pk48), n, _np_ptr(msgs), msgs.shape[1], _np_ptr(sigs), _np_ptr(st), threads)
    return st


def beacon_message(prev_sig, prev_round, rnd):
    out = ctypes.create_string_buffer(32)
    lib().twin_beacon_message(_buf(prev_sig), len(prev_sig), prev_round, rnd, out)
    return out.raw


def gen_chain(sk, seed, first_round, n):
    out = np.zeros((n, 96), dtype=np.uint8)
    lib().twin_gen_chain(_buf(int(sk).to_bytes(32, "big")), _buf(seed), len(seed), first_round, n, _np_ptr(out))
    return out


def pubpoly_eval(commits, index):
    cb = b"".join(commits)
    out = ctypes.create_string_buffer(48)
    st = lib().twin_pubpoly_eval(_buf(cb), len(commits), index, out)
    return st, out.raw


def g1_mul_gen(sk):
    out = ctypes.create_string_buffer(48)
    lib().twin_g1_mul_gen(_buf(int(sk).to_bytes(32, "big")), out)
    return out.raw


def verify_partial(commits, msg, partial):
    cb = b"".join(commits)
    return lib().twin_verify_partial(_buf(cb), len(commits), _buf(msg), len(msg), _buf(partial), len(partial))


def recover(commits, msg, partials, t, n):
    cb = b"".join(commits)
    pb = b"".join(partials)
    out = ctypes.create_string_buffer(96)
    ss = ctypes.create_string_buffer(len(partials))
    rs = lib().twin_recover(_buf(cb), t, n, _buf(msg), len(msg), _buf(pb), len(partials), out, ss)
    return (out.raw if rs == 0 else None), rs, list(ss.raw)


def recover_batch(commits, t, n, msgs32, partials98, threads=1):
    """msgs32 (R, 32), partials98 (R, k, 98) -> (sigs (R,96), round_status (R,), share_status (R,k))."""
    cb = b"".join(commits)
    msgs32 = np.ascontiguousarray(msgs32, dtype=np.uint8)
    partials98 = np.ascontiguousarray(partials98, dtype=np.uint8)
    R_, k = partials98.shape[0], partials98.shape[1]
    out = np.zeros((R_, 96), dtype=np.uint8)
    rs = np.zeros(R_, dtype=np.uint8)
    ss = np.zeros((R_, k), dtype=np.uint8)
    lib().twin_recover_batch(_buf(cb), t, n, R_, _np_ptr(msgs32), _np_ptr(partials98), k, _np_ptr(out), _np_ptr(rs),
                             _np_ptr(ss), threads)
    return out, rs, ss


def set_dst(dst=None):
    """The DST of twin sign / verify / recover (None: BLS_SIG_..._NUL_)."""
    if dst is None:
        lib().twin_set_dst(None, 0)
    else:
        lib().twin_set_dst(_buf(dst), len(dst))


def c1_batch(commits, t, n, shares, msgs32, threads=1):
    """BASELINE configs[0] per round: n Signs + Recover + VerifyRecovered -> (sigs (R, 96), rounds verified)."""
    cb = b"".join(commits)
    sb = b"".join(int(v).to_bytes(32, "big") for v in shares)
    msgs32 = np.ascontiguousarray(msgs32, dtype=np.uint8)
    R_ = msgs32.shape[0]
    out = np.zeros((R_, 96), dtype=np.uint8)
    ok = lib().twin_c1_batch(_buf(cb), t, n, _buf(sb), R_, _np_ptr(msgs32), _np_ptr(out), threads)
    return out, int(ok)


def pairing_cubed(g1_48, g2_96):
    out = ctypes.create_string_buffer(576)
    st = lib().twin_pairing_cubed(_buf(g1_48), _buf(g2_96), out)
    return st, out.raw
