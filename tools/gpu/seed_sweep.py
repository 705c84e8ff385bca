"""Diagnostic: batch-path verdict of the 100k-round bench batch for a range of seeds."""
import ctypes
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from drand_amd import _lib as L  # noqa: E402
from drand_amd import tbls  # noqa: E402
from tools import synthetic as S  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 100000
seeds = list(range(int(sys.argv[2]), int(sys.argv[3]))) if len(sys.argv) > 3 else list(range(15, 30))
reps = int(os.environ.get("SWEEP_REPS", "1"))
seeds = [1000, 1001, 7] + seeds * reps
lib = L.lib(0)
mm = np.memmap(os.path.join(ROOT, "data", "chain_v1_100000.bin"), dtype=np.uint8, mode="r", shape=(100000, 96))
sigs = np.array(mm[:n])
rounds = np.arange(1, n + 1, dtype=np.uint64)
prev = [S.GENESIS_SEED] + [bytes(sigs[i]) for i in range(n - 1)]
_, _, psb, off = tbls._beacon_arrays(rounds - 1, rounds, prev)
dev = torch.device("cuda", 0)
d_pr = torch.from_numpy((rounds - 1).astype(np.int64)).to(dev)
d_r = torch.from_numpy(rounds.astype(np.int64)).to(dev)
d_ps = torch.from_numpy(psb).to(dev)
d_off = torch.from_numpy(off.astype(np.int32)).to(dev)
d_sig = torch.from_numpy(sigs).to(dev)
d_st = torch.zeros(n, dtype=torch.uint8, device=dev)
if os.environ.get("SWEEP_TIMING"):
    L.check(lib.dg_set_timing(1))
for seed in seeds:
    t0 = time.time()
    L.check(lib.dg_verify_beacons_dev(ctypes.c_char_p(S.GROUP_PK), n, L.ptr(d_pr), L.ptr(d_r), L.ptr(d_ps), L.ptr(d_off),
                                      L.ptr(d_sig), L.ptr(d_st), seed, None))
    ok, iso = L.last_batch_flags()
    print("seed", seed, "batch_ok", ok, "iso", iso, "bad", int((d_st != 0).sum().item()), "%.1f ms" % ((time.time() - t0) * 1e3),
          flush=True)
