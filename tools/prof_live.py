"""Per-kernel anatomy of one live-round call (tooling): bench.py's live_latency inputs (one round, n = 64, t = 33),
dg_recover through the host-buffer API, per-kernel HIP-event timings (dg_set_timing) of one call after warmup, sorted
by total time, and the call's wall time with and without the timing events.

    python tools/prof_live.py [--reps 20]
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    import bench
    from drand_amd import _lib as L
    from drand_amd import tbls

    L.lib(0)
    t, n = 33, 64
    src = bench.RoundSource(tbls, 1000)
    pub, _, _, msgs, parts = bench.make_group_rounds(tbls, src, 1, 8, t, n)
    m1, p1 = msgs[:1], parts[:1]
    calls = {"recover_full": lambda: tbls.recover_batch(pub, m1, p1, t, n),
             "verify_recovered": lambda: tbls.verify_recovered_batch(pub.commit(), m1, src.sigs[:1])}
    for name, fn in calls.items():
        for _ in range(3):
            fn()
        t0 = time.perf_counter()
        for _ in range(a.reps):
            fn()
        wall = (time.perf_counter() - t0) / a.reps * 1e3
        L.check(L.lib().dg_set_timing(1))
        fn()
        kt = L.timings()
        L.check(L.lib().dg_set_timing(0))
        tot = sum(us * k for us, k in kt.values())
        print("%s: %.2f ms per call; %d kernels, %.2f ms of kernel time (events)" % (name, wall, sum(k for _, k in
                                                                                             kt.values()), tot / 1e3))
        for k, (us, c) in sorted(kt.items(), key=lambda x: -x[1][0] * x[1][1])[:25]:
            print("   %-24s %4d x %9.1f us = %8.1f us" % (k, c, us, us * c))


if __name__ == "__main__":
    main()
