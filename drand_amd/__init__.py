"""drand_amd: MI355X-native threshold-BLS verification/aggregation for drand (BLS12-381, gfx950).

The product is the C-ABI library libdrandgpu.so (include/drand_gpu.h); `tbls` mirrors kyber's
sign.ThresholdScheme as drand uses it through key.Scheme (key/curve.go:30) and `beacon` the chain
helpers of beacon/chain.go, both as thin ctypes callers of that library.
"""
from . import _lib  # noqa: F401

__all__ = ["tbls", "beacon"]
