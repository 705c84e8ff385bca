"""Generate the synthetic linked beacon chain sigma_1..sigma_N with the CPU twin (fixture generation).

sigma_r = x * H(Message(sigma_{r-1}, r-1, r)), sigma_0 = the genesis seed (beacon/chain.go:86-94,
beacon/beacon.go:108-112).  The chain is inherently sequential (~2.5 ms/round on one host core),
so it is generated once here and shipped to the GPU box as data/chain_v1_<N>.bin (git-ignored,
not gpurun-ignored).  Usage: python tools/gen_chain.py N [--from-prefix existing.bin]
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from oracle import twin  # noqa: E402
from tools import synthetic as S  # noqa: E402


def main():
    n = int(sys.argv[1])
    out = S.chain_path(n)
    os.makedirs(os.path.dirname(out), exist_ok=True)
    tmp = out + ".partial"
    done = 0
    if not os.path.exists(tmp):
        # every chain file is a prefix of the longer ones: start from the longest shorter one
        d = os.path.dirname(out)
        have = sorted((int(f.split("_")[-1].split(".")[0]), f) for f in os.listdir(d)
                      if f.startswith("chain_v1_") and f.endswith(".bin"))
        have = [(m, f) for m, f in have if m < n]
        if have:
            import shutil
            shutil.copyfile(os.path.join(d, have[-1][1]), tmp)
    if os.path.exists(tmp):
        done = os.path.getsize(tmp) // 96
    x = S.master_secret()
    t0 = time.time()
    with open(tmp, "ab") as f:
        while done < n:
            k = min(5000, n - done)
            if done == 0:
                prev = S.GENESIS_SEED
            else:
                with open(tmp, "rb") as g:
                    g.seek((done - 1) * 96)
                    prev = g.read(96)
            sigs = twin.gen_chain(x, prev, done + 1, k)
            f.write(sigs.tobytes())
            f.flush()
            done += k
            print("rounds %d/%d  %.1f s" % (done, n, time.time() - t0), flush=True)
    os.replace(tmp, out)


if __name__ == "__main__":
    main()
