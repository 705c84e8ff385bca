"""Deterministic corruption of partial signatures (BASELINE config C5 modes).

No curve arithmetic here: modes that need a fresh signature take it from the caller (`resign`), so the
same helper serves the GPU bench (resign = dg_sign) and the tests (resign = the CPU twin).
"""
import hashlib

MODES = ["wrong_scalar", "other_round", "index_rewritten", "random_bytes", "bitflip_x", "infinity"]


def corrupt_batch(partials, items, n_shares, resign):
    """partials: (R, k, 98) uint8 array (modified in place); items: list of (r, j, mode).
    resign(list of (share_index, scalar_delta, round_delta)) -> list of 96 B signatures, where the signature
    is of share `share_index` with its scalar + scalar_delta on the message of round r + round_delta."""
    need = [(r, j, m) for r, j, m in items if m in ("wrong_scalar", "other_round")]
    reqs = []
    for r, j, m in need:
        idx = int(partials[r, j, 0]) << 8 | int(partials[r, j, 1])
        reqs.append((r, idx, 1 if m == "wrong_scalar" else 0, 0 if m == "wrong_scalar" else 1))
    fresh = resign(reqs) if reqs else []
    fi = 0
    for r, j, m in items:
        p = partials[r, j]
        idx = int(p[0]) << 8 | int(p[1])
        if m in ("wrong_scalar", "other_round"):
            p[2:] = list(fresh[fi])
            fi += 1
        elif m == "index_rewritten":
            nidx = (idx + 1) % n_shares
            p[0], p[1] = nidx >> 8, nidx & 0xFF
        elif m == "random_bytes":
            p[2:] = list(hashlib.sha256(b"rnd/%d/%d" % (r, j)).digest() * 3)
        elif m == "bitflip_x":
            p[2 + 40] ^= 0x04
        elif m == "infinity":
            p[2] = 0xC0
            p[3:] = 0
        else:
            raise ValueError(m)
    return partials


def pick(R, k, frac, seed=b"c5"):
    """Deterministic ~frac of (round, share) cells with cycling modes."""
    out = []
    c = 0
    for r in range(R):
        for j in range(k):
            h = hashlib.sha256(seed + r.to_bytes(8, "big") + j.to_bytes(4, "big")).digest()
            if int.from_bytes(h[:4], "big") < frac * 2**32:
                out.append((r, j, MODES[c % len(MODES)]))
                c += 1
    return out
