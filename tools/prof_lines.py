"""Profiling driver (tooling): the calls of ONE bench.py sub-line alone, so that a rocprofv3 --pmc pass's per-kernel
averages belong to one workload (bench.py runs Recover and VerifyPartial of all partials in one process, and C5's
Recover beside its VerifyPartial line, which share kernels).  Inputs are bench.py's own (make_group_rounds,
make_c5_inputs), resident in HBM; one warmup call, then --calls timed calls.

    python tools/prof_lines.py c3     # dg_recover_dev, n = 64, t = 33, 100k rounds (bench.py `recover`)
    python tools/prof_lines.py c3vp   # dg_verify_partials_dev over all 100k x 64 partials (`c2_verify_all`)
    python tools/prof_lines.py c5     # dg_recover_dev, n = 256, t = 129, 10k rounds, 10% corrupted (`adversarial`)
    python tools/prof_lines.py c5vp   # dg_verify_partials_dev over C5's corrupted set (`vp_negative`)
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("line", choices=["c3", "c3vp", "c5", "c5vp"])
    ap.add_argument("--rounds", type=int, default=0, help="default: the bench line's (100k for c3*, 10k for c5*)")
    ap.add_argument("--calls", type=int, default=1)
    a = ap.parse_args()
    import numpy as np
    import torch

    import bench
    from drand_amd import _lib as L
    from drand_amd import shard, tbls

    L.lib(0)
    dev = torch.device("cuda", 0)
    if a.line.startswith("c3"):
        R, t, n = a.rounds or 100000, 33, 64
        src = bench.RoundSource(tbls, R)
        pub, _, _, msgs, parts = bench.make_group_rounds(tbls, src, 1, R, t, n)
    else:
        R, t, n = a.rounds or 10000, 129, 256
        src = bench.RoundSource(tbls, R + 1)
        pub, _, msgs, parts, _, _, _, _, _, _ = bench.make_c5_inputs(tbls, shard, src, R, 1, 0, t, n)
    d_msgs = torch.from_numpy(np.ascontiguousarray(msgs)).to(dev)
    d_parts = torch.from_numpy(np.ascontiguousarray(parts)).to(dev)
    if a.line in ("c3", "c5"):
        call = lambda s: tbls.recover_batch_dev(pub, d_msgs, d_parts, t, n, seed=s)  # noqa: E731
    else:
        call = lambda s: tbls.verify_partial_batch_dev(pub, d_msgs, d_parts, seed=s)  # noqa: E731
    call(1)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for s in range(a.calls):
        call(2 + s)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / a.calls
    print("%s: %d rounds, %.1f ms per call, %.0f rounds/s" % (a.line, R, dt * 1e3, R / dt), flush=True)


if __name__ == "__main__":
    main()
