"""One blocking 100k-round batch with 1% of the signatures replaced (bench.py's c2_negative positions), run `reps`
times with nothing else on the GPU: the isolation kernels' latency without concurrent bulk work (tooling, for
rocprofv3 --kernel-trace).   python tools/trace/neg_single.py [reps]"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from drand_amd import _lib as L  # noqa: E402
from tools import synthetic as S  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    N = 100000
    n_, path_ = S.find_chain(N)
    sigs = np.fromfile(path_, dtype=np.uint8).reshape(n_, 96)[:N]
    bad_pos = np.unique((np.arange(N // 100, dtype=np.int64) * 7919 + 13) % N)
    bad = sigs.copy()
    bad[bad_pos] = sigs[np.where(bad_pos + 1 < N, bad_pos + 1, bad_pos - 1)]
    rounds = np.arange(1, N + 1, dtype=np.uint64)
    prev = np.concatenate([np.frombuffer(S.GENESIS_SEED, np.uint8), sigs[:-1].reshape(-1)])
    off = np.concatenate([[0], 32 + 96 * np.arange(N, dtype=np.int64)]).astype(np.int32)
    dev = torch.device("cuda", 0)
    d = [torch.from_numpy(a).to(dev) for a in ((rounds - 1).astype(np.int64), rounds.astype(np.int64), prev, off, bad)]
    st = torch.full((N,), 99, dtype=torch.uint8, device=dev)
    lib = L.lib(0)
    for r in range(reps):
        L.check(lib.dg_verify_beacons_dev(S.GROUP_PK, N, L.ptr(d[0]), L.ptr(d[1]), L.ptr(d[2]), L.ptr(d[3]),
                                          L.ptr(d[4]), L.ptr(st), 77 + r, None))
        torch.cuda.synchronize()
        got = st.cpu().numpy()
        assert np.nonzero(got)[0].tolist() == bad_pos.tolist()
    print("ok", reps)


if __name__ == "__main__":
    main()
