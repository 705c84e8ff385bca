"""ctypes binding of libdrandgpu.so (the C-ABI of include/drand_gpu.h).

The library is built in-tree by __graft_entry__.build() (hipcc --offload-arch=gfx950).  There is no
CPU fallback: if the library or a gfx950 device is missing, every call raises DrandGpuError.
"""
import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("DRAND_GPU_LIB", os.path.join(_HERE, "libdrandgpu.so"))

# status codes (include/drand_gpu.h)
ST_OK = 0
ST_BAD_SIG = 1
ST_SIG_DECODE = 2
ST_BAD_INDEX = 3
ST_PK_DECODE = 4
ST_NOT_ENOUGH = 5
ST_NOT_EXAMINED = 255

DST_NUL = b"BLS_SIG_BLS12381G2_XMD:SHA-256_SSWU_RO_NUL_"

# Every entry point the header declares, with ctypes signatures.
_P = ctypes.c_void_p
_SZ = ctypes.c_size_t
_U32 = ctypes.c_uint32
_U64 = ctypes.c_uint64
_I = ctypes.c_int
SIGNATURES = {
    "dg_init": ([_I], _I),
    "dg_shutdown": ([], None),
    "dg_last_error": ([], ctypes.c_char_p),
    "dg_device_ready": ([], _I),
    "dg_hash_to_g2": ([_SZ, _P, _SZ, _P, _SZ, _P], _I),
    "dg_sign": ([_SZ, _P, _P, _P, _SZ, _P], _I),
    "dg_verify": ([_P, _SZ, _P, _SZ, _P, _P, _U64], _I),
    "dg_verify_beacons": ([_P, _SZ, _P, _P, _P, _P, _P, _P, _U64], _I),
    "dg_check_links": ([_U64, _P, _SZ, _SZ, _P, _P, _P, _P, _P, _P], _I),
    "dg_beacon_messages": ([_SZ, _P, _P, _P, _P, _P], _I),
    "dg_randomness": ([_SZ, _P, _P], _I),
    "dg_pubpoly_eval": ([_P, _U32, _SZ, _P, _P], _I),
    "dg_verify_partials": ([_P, _U32, _SZ, _P, _SZ, _U32, _P, _P, _U64], _I),
    "dg_recover": ([_P, _U32, _U32, _SZ, _P, _SZ, _U32, _P, _P, _P, _P, _U64], _I),
    "dg_recover_verified": ([_U32, _U32, _SZ, _U32, _P, _P, _P, _P, _P], _I),
    "dg_set_hash_dst": ([_P, _SZ], _I),
    "dg_get_hash_dst": ([_P, _SZ, _P], _I),
    "dg_verify_beacons_dev": ([_P, _SZ, _P, _P, _P, _P, _P, _P, _U64, _P], _I),
    "dg_verify_beacons_dev_async": ([_P, _SZ, _P, _P, _P, _P, _P, _P, _U64, _P, _P], _I),
    "dg_wait_all": ([], _I),
    "dg_queue_plan": ([_I, _P, _P], _I),
    "dg_last_batch_stream": ([_P], _I),
    "dg_last_batch_flags": ([_P], _I),
    "dg_fallback_count": ([_P], _I),
    "dg_group_counts": ([_P], _I),
    "dg_isolation_counts": ([_P], _I),
    "dg_set_group_size": ([_U32], _I),
    "dg_recover_dev": ([_P, _U32, _U32, _SZ, _P, _SZ, _U32, _P, _P, _P, _P, _U64], _I),
    "dg_verify_partials_dev": ([_P, _U32, _SZ, _P, _SZ, _U32, _P, _P, _U64], _I),
    "dg_recover_verified_dev": ([_U32, _U32, _SZ, _U32, _P, _P, _P, _P, _P], _I),
    "dg_set_timing": ([_I], _I),
    "dg_last_timings": ([_P, _P, _P, _I], _I),
}


class DrandGpuError(RuntimeError):
    pass


_lib = None
_device = None


def load():
    """Load the shared library (no device needed).  Raises if it was not built."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise DrandGpuError("libdrandgpu.so not built: run __graft_entry__.build() (hipcc, gfx950)")
        lib = ctypes.CDLL(LIB_PATH)
        for name, (args, res) in SIGNATURES.items():
            fn = getattr(lib, name)
            fn.argtypes = args
            fn.restype = res
        _lib = lib
    return _lib


def hw_queues():
    """GPU_MAX_HW_QUEUES as the C environment holds it (libdrandgpu.so sets its default there at load time, which
    os.environ, copied at interpreter start, does not see); HIP's own default 4 if unset."""
    libc = ctypes.CDLL(None)
    libc.getenv.restype = ctypes.c_char_p
    v = libc.getenv(b"GPU_MAX_HW_QUEUES")
    return int(v) if v else 4


def lib(device=None):
    """The library with a device selected (LOCAL_RANK, else 0)."""
    global _device
    L = load()
    if device is None:
        device = int(os.environ.get("LOCAL_RANK", "0")) if _device is None else _device
    if _device != device:
        check(L.dg_init(device))
        _device = device
    return L


def check(rc):
    if rc != 0:
        msg = load().dg_last_error()
        raise DrandGpuError("libdrandgpu error %d: %s" % (rc, msg.decode() if msg else ""))
    return rc


def ptr(a):
    if a is None:
        return None
    if isinstance(a, np.ndarray):
        return a.ctypes.data_as(ctypes.c_void_p)
    if isinstance(a, (bytes, bytearray)):
        return ctypes.cast(ctypes.c_char_p(bytes(a)), ctypes.c_void_p)
    if hasattr(a, "data_ptr"):  # torch tensor (device-resident API)
        return ctypes.c_void_p(a.data_ptr())
    raise TypeError(type(a))


def u8(a, shape=None):
    """bytes / list of bytes / ndarray -> contiguous uint8 ndarray."""
    if isinstance(a, np.ndarray):
        arr = np.ascontiguousarray(a, dtype=np.uint8)
    elif isinstance(a, (bytes, bytearray)):
        arr = np.frombuffer(bytes(a), dtype=np.uint8).copy()
    else:
        def flat(x):
            if isinstance(x, (bytes, bytearray, memoryview)):
                return bytes(x)
            if isinstance(x, np.ndarray):
                return np.ascontiguousarray(x, dtype=np.uint8).tobytes()
            return b"".join(flat(y) for y in x)

        arr = np.frombuffer(flat(a), dtype=np.uint8).copy()
    if shape is not None:
        arr = arr.reshape(shape)
    return arr


def last_batch_flags():
    """(batch equation held, some item isolated) for the most recent verification batch."""
    out = np.zeros(2, dtype=np.uint32)
    check(lib().dg_last_batch_flags(ptr(out)))
    return bool(out[0]), bool(out[1])


def fallback_count():
    """Batches since dg_init that ran the per-item pass (batch equation failed or items isolated)."""
    out = np.zeros(1, dtype=np.uint64)
    check(lib().dg_fallback_count(ptr(out)))
    return int(out[0])


def group_counts():
    """Recover's per-item pass since dg_init: [checks of 1, 2, 3, 4 shares of a round at once]."""
    out = np.zeros(4, dtype=np.uint64)
    check(lib().dg_group_counts(ptr(out)))
    return [int(v) for v in out]


def isolation_counts():
    """The cross-round isolation of failed single-key batches since dg_init (xr.h): [group tests of 4 quads, tests
    of one quad (4 rounds), single rounds]."""
    out = np.zeros(3, dtype=np.uint64)
    check(lib().dg_isolation_counts(ptr(out)))
    return [int(v) for v in out]


def timings():
    """Per-kernel average launch time (us) accumulated since dg_set_timing(1)."""
    L = load()
    cap = 256
    names = (ctypes.c_char_p * cap)()
    us = (ctypes.c_double * cap)()
    launches = (ctypes.c_int * cap)()
    k = L.dg_last_timings(ctypes.cast(names, _P), ctypes.cast(us, _P), ctypes.cast(launches, _P), cap)
    return {names[i].decode(): (us[i], launches[i]) for i in range(k)}
