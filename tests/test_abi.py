"""The C-ABI boundary (CPU): libdrandgpu.so loads, exports every function include/drand_gpu.h declares
with the argument count the ctypes binding uses, and refuses compute without a gfx950 device (no CPU
fallback exists)."""
import os
import re
import subprocess
import sys

import numpy as np
import pytest

from drand_amd import _lib as L

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "drand_gpu.h")


def declared():
    txt = open(HEADER).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    out = {}
    for m in re.finditer(r"\b(?:int|void|const char\*)\s+(dg_\w+)\s*\(([^)]*)\)\s*;", txt):
        args = m.group(2).strip()
        n = 0 if args in ("", "void") else args.count(",") + 1
        out[m.group(1)] = n
    return out


def test_header_declares_the_survey_boundary():
    d = declared()
    for name in ("dg_init", "dg_shutdown", "dg_verify", "dg_verify_beacons", "dg_verify_partials", "dg_recover",
                 "dg_hash_to_g2", "dg_sign", "dg_pubpoly_eval", "dg_check_links", "dg_beacon_messages",
                 "dg_randomness"):
        assert name in d, name


def test_library_exports_every_declared_symbol():
    lib = L.load()
    nm = subprocess.run(["nm", "-D", "--defined-only", L.LIB_PATH], capture_output=True, text=True, check=True).stdout
    exported = set(re.findall(r"\bT (dg_\w+)", nm))
    d = declared()
    assert set(d) <= exported, set(d) - exported
    for name, nargs in d.items():
        assert hasattr(lib, name)
        assert name in L.SIGNATURES, name
        assert len(L.SIGNATURES[name][0]) == nargs, name


def test_no_device_means_no_compute():
    import torch

    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    lib = L.load()
    assert lib.dg_device_ready() == 0
    out = np.zeros(96, np.uint8)
    msg = np.zeros(32, np.uint8)
    rc = lib.dg_hash_to_g2(1, L.ptr(msg), 32, L.ptr(L.DST_NUL), len(L.DST_NUL), L.ptr(out))
    assert rc == -1  # DG_E_NODEV: there is no CPU fallback
    assert b"gfx950" in lib.dg_last_error()
    with pytest.raises(L.DrandGpuError):
        from drand_amd import tbls

        tbls.hash_to_g2([bytes(32)])


NATIVE = os.path.join(ROOT, "tests", "native")


def test_cpp_caller_compiles_against_the_header_and_runs_sanitized():
    """tests/native/abi_caller.cpp binds every entry point to a function pointer of the exact C type (so a
    header / library signature drift breaks the build, as it would break cgo), then calls each once without a
    device under ASan + UBSan: compute calls return DG_E_NODEV, host-only state (timing, DST) works."""
    src = open(os.path.join(NATIVE, "abi_caller.cpp")).read()
    missing = [n for n in declared() if "EXPECT_TYPE(%s," % n not in src]
    assert missing == [], missing
    subprocess.run(["make", "-s", "-C", NATIVE, "abi_caller"], check=True)
    r = subprocess.run([os.path.join(NATIVE, "abi_caller")], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and "abi_caller: ok" in r.stdout, r.stdout + r.stderr


def test_host_arithmetic_under_asan_ubsan():
    """The kernels' device arithmetic built for the host with AddressSanitizer and UBSan (no recovery): the
    word-wise expansion, both phase pipelines, decode round trips and the safegcd inversion run clean."""
    subprocess.run(["make", "-s", "-C", NATIVE, "hostcheck_san"], check=True)
    r = subprocess.run([os.path.join(NATIVE, "hostcheck_san")], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "hostcheck_san: ok" in r.stdout, r.stdout + r.stderr


def test_prewarmed_kernels_hold_the_largest_private_segment():
    """dg_init dispatches every kernel that may run on a stream there once with no work, largest private segment
    first (read at run time with hipFuncGetAttributes), so each queue's scratch reaches its final size before any batch
    runs (a larger private segment needed later regrows the queue's scratch mid-pipeline: stalls, or
    HSA_STATUS_ERROR_OUT_OF_RESOURCES).  From the gfx950 code-object metadata of the built objects: no kernel exceeds
    6 KB of private segment (the round-3 per-item kernels held ~15 KB and failed dg_init at 8 queues); the two
    largest, k_sign and k_hash_to_g2, are the fixture kernels of the fb stream, so every workspace queue reserves less;
    and the workspace streams' prewarm list holds the largest private segment of the rest."""
    import re
    import tempfile

    from tools import resource_usage as RU

    tus = ("drand_gpu.o", "kernels_hot.o") + tuple("kernels_check_%s.o" % p for p in "abcdef")
    objs = [os.path.join(ROOT, "drand_amd", "csrc", t) for t in tus]
    if not all(os.path.exists(o) for o in objs):
        pytest.skip("library objects not built")
    with tempfile.TemporaryDirectory() as tmp:
        ks = {k[".name"]: int(k.get(".private_segment_fixed_size", 0)) for o in objs for k in RU.kernels_of(o, tmp)}
    assert max(ks.values()) <= 6144, sorted(ks.items(), key=lambda x: -x[1])[:4]
    fb = ("k_sign", "k_hash_to_g2")
    rest = {k: v for k, v in ks.items() if k not in fb}
    assert min(ks[k] for k in fb) >= max(rest.values()), sorted(ks.items(), key=lambda x: -x[1])[:4]
    src = open(os.path.join(ROOT, "drand_amd", "csrc", "drand_gpu.hip")).read()
    block = src[src.index("const std::vector<Warm> on_sets"):src.index("const std::vector<Warm> on_fb")]
    warmed = set(re.findall(r"\(const void\*\)(k_\w+)", block))
    assert warmed <= set(ks), warmed - set(ks)
    # the largest kernel dg_init prewarms on the workspace streams holds the largest private segment of every kernel
    # that runs there (so no later dispatch regrows a workspace queue's scratch)
    assert max(ks[k] for k in warmed) == max(rest.values()), sorted(rest.items(), key=lambda x: -x[1])[:4]


_QUEUES_CHILD = r"""
import sys
sys.path.insert(0, sys.argv[1])
from drand_amd import _lib as L
L.load()
print(L.hw_queues())
"""


@pytest.mark.parametrize("preset,want", [(None, 16), ("4", 4), ("24", 24)])
def test_library_load_sets_the_default_hw_queue_count(preset, want):
    """Loading libdrandgpu.so asks HIP for 16 hardware queues (GPU_MAX_HW_QUEUES, read when the runtime starts) unless
    the process chose a value: the default a drand process gets without reading INTEGRATION.md (no device needed)."""
    env = {k: v for k, v in os.environ.items() if k != "GPU_MAX_HW_QUEUES"}
    if preset is not None:
        env["GPU_MAX_HW_QUEUES"] = preset
    r = subprocess.run([sys.executable, "-c", _QUEUES_CHILD, ROOT], env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    assert int(r.stdout.strip().splitlines()[-1]) == want


def test_queue_plan():
    """dg_queue_plan (drand_gpu.hip queue_plan): 10 sets from 12 hardware queues up; between 5 and 11
    queues, queues - 2 sets, so no two library streams share a queue; at 4 queues or fewer a multiple of the queue
    count.  The per-item pass (the check pipeline) runs on the set streams at every queue count."""
    import ctypes

    lib = L.load()
    got = {}
    for q in range(0, 33):
        sets, shared = ctypes.c_int(), ctypes.c_int()
        assert lib.dg_queue_plan(q, ctypes.byref(sets), ctypes.byref(shared)) == 0
        got[q] = (sets.value, shared.value)
    assert got[0] == got[4] == (8, 1)  # HIP's default when unset
    assert got[1] == (10, 1) and got[2] == (10, 1) and got[3] == (9, 1)
    for q in range(5, 12):
        assert got[q] == (q - 2, 1)
    for q in range(12, 33):
        assert got[q] == (10, 1)
    for q in range(1, 5):
        assert got[q][0] % q == 0


def test_release_build_reads_no_retired_switches():
    """Round-4 verdict (hygiene): DG_NO_BIND (and the removed A/B switches, round 6's DG_XR_SKIP among them) have no
    effect on the release build -- the library never reads them, so their names are absent from its strings (getenv
    takes the name as a literal)."""
    blob = open(L.LIB_PATH, "rb").read()
    for name in (b"DG_NO_BIND", b"DG_CK_OLD", b"DG_FUSED", b"DG_MSM_JAC", b"DG_FP2_LAZY", b"DG_FP6_DIG",
                 b"DG_SUB_SEPARATE", b"DG_XR_SKIP", b"DG_STAGGER", b"DG_GRAPH", b"DG_SET_ORDER"):
        assert name not in blob, name
