"""Per-kernel times of one dg_recover batch (BASELINE configs[2]: n = 64, t = 33)."""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from drand_amd import _lib as L  # noqa: E402
from drand_amd import tbls  # noqa: E402

R = int(sys.argv[1]) if len(sys.argv) > 1 else 20000
chain = bench.load_chain(R + 1)
lib = L.lib(0)
t0 = time.time()
bench.recover_bench(L, tbls, chain, 1, R, 33, 64, 1)
print("recover bench %.1f s" % (time.time() - t0))
L.check(lib.dg_set_timing(1))
from tools import synthetic as S  # noqa: E402
g = json.load(open(os.path.join(ROOT, "tests", "golden", "groups.json")))["t33"]
pub = tbls.PubPoly([bytes.fromhex(c) for c in g])
coeffs = S.poly_coeffs(33)
shares = [S.share_value(coeffs, i) for i in range(64)]
rounds = np.arange(1, R + 1, dtype=np.uint64)
prev = [bytes(chain[r - 2]) if r >= 2 else S.GENESIS_SEED for r in rounds.tolist()]
msgs = tbls.beacon_messages(rounds - 1, rounds, prev)
parts = tbls.sign_batch([shares[i] for _ in range(R) for i in range(64)], np.repeat(msgs, 64, axis=0),
                        [i for _ in range(R) for i in range(64)]).reshape(R, 64, 98)
L.check(lib.dg_set_timing(0))
L.check(lib.dg_set_timing(1))
t0 = time.time()
tbls.recover_batch(pub, msgs, parts, 33, 64, seed=3)
dt = time.time() - t0
kt = L.timings()
print("recover %.1f ms" % (dt * 1e3))
for k, (us, n) in sorted(kt.items(), key=lambda kv: -kv[1][0] * kv[1][1]):
    print("%-22s %9.1f us x %d" % (k, us, n))
