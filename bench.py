"""Benchmark of the threshold-BLS hot path (BASELINE.json): verified beacon rounds/s, Recover/s at n = 64.

A step = one pass of beacon.VerifyBeacon (beacon/chain.go:65-71) over this rank's contiguous range of the
synthetic linked chain, in device-resident batches of at most --batch rounds (beacon.Message on the device,
hash-to-G2, sigma decode with a batched subgroup check, RLC multi-pairing with one shared final
exponentiation; asynchronous, so one batch's latency-bound tail overlaps the next batch's head), then the
RCCL all-gather of the per-round verdict bitmaps.

    N = 1 (default): BASELINE configs[1], 100k rounds per step, one shared group key.
    N > 1:           BASELINE configs[3], the 1M-round chain per step sharded into N contiguous ranges
                     (strong scaling; --global-rounds overrides the total at any N).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--global-rounds R] [--no-cpu-baseline]

--gpus N without a torchrun environment starts the N ranks itself (torch.distributed.run as a child
process, before anything touches the GPU) and exits with their status; a rank whose WORLD_SIZE differs
from --gpus exits non-zero.  Rank 0 prints ONE JSON line (contract in the task statement), kept under
~4 KB so the driver's record holds all of it.  Beside the headline it carries the Recover lines
(configs[2] C3 and configs[4] C5, sharded the same way, their outputs all-gathered), the live-round
latency lines, the syncFrom catch-up line, the CPU baselines (rank 0, at every N,
after the GPU timed regions, on every host core this process may use) and the roofline objects:
algorithmic multiply-adds of the dominant kernel (profiles/opcounts.json: 300 per Montgomery product,
BASELINE.md) over its HIP-event launch time, against the v_mad_u64_u32 peak each rank measures on its own
GPU (tools/microbench/probe.hip).  The per-kernel timing tables go to a side file (--tables-out).
"""
import argparse
import collections
import ctypes
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from tools import synthetic as S  # noqa: E402

METRIC = "verified beacon rounds/sec (pairing checks/s)"


def log(*a):
    print("[bench]", *a, file=sys.stderr, flush=True)


def host_cores():
    """The host cores for the CPU baselines: every CPU this process may run on (its affinity mask, capped by
    a cgroup CPU quota when one is set -- threads beyond the quota only time-slice), not OMP_NUM_THREADS.
    Returns (threads used, CPUs of the machine, cgroup quota in CPUs or None)."""
    aff = len(os.sched_getaffinity(0))
    quota = None
    try:
        q, p = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = int(q) / int(p)
    except (OSError, ValueError):
        pass
    use = aff if quota is None else max(1, min(aff, int(quota)))
    return use, os.cpu_count() or use, quota


def cpu_label(cb, threads, machine, quota):
    """The core-count fields of a cpu_baseline object: the threads used and the machine's CPU count, and a
    linear estimate for all of the machine's CPUs when the process was held to fewer of them."""
    cb["cores"] = threads
    cb["host_cpus"] = machine
    if quota is not None:
        cb["cgroup_cpu_quota"] = quota
    if machine > threads:
        cb["all_host_cpus_linear_est"] = cb["value"] * machine / threads
    return cb


def traffic_of(kernel, config="head"):
    """HBM-side bytes per launch of `kernel` from the committed PMC passes (profiles/traffic.json, made by
    tools/traffic.py from separate rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE runs of this bench; config "head",
    "c3" or "c5"): 2 x FETCH_SIZE + WRITE_SIZE (the gfx950 correction of FETCH_SIZE), or None without a
    profile."""
    p = os.path.join(ROOT, "profiles", "traffic.json")
    if not os.path.exists(p):
        return None
    t = json.load(open(p)).get("configs", {}).get(config, {}).get(kernel)
    return t["bytes_per_launch"] if t else None


def load_chain(total, data_dir=None):
    """sigs (total, 96) of rounds 1..total of the synthetic linked chain: the smallest chain file that holds them,
    checked against its pinned SHA-256 (tools/synthetic.CHAIN_SHA256).  None when no file covers `total` (or the
    covering file fails its digest: logged)."""
    try:
        n, path = S.find_chain(total, data_dir)
    except S.ChainFileError as e:
        log("chain:", e)
        return None
    mm = np.memmap(path, dtype=np.uint8, mode="r", shape=(n, 96))
    return np.array(mm[:total])


def require_chain(total, allow_unlinked, data_dir=None):
    """The chain rounds a timed line verifies.  Without a pinned chain file that covers them the bench exits
    non-zero (status 3) unless --allow-unlinked was given: a configs[1]/[3] line must never silently turn into
    unlinked rounds signed by the library under test."""
    chain = load_chain(total, data_dir)
    if chain is None and not allow_unlinked:
        log("no digest-pinned chain file covers %d rounds: refusing to measure unlinked GPU-signed rounds "
            "(--allow-unlinked overrides; tools/gen_chain.py %d makes the file)" % (total, total))
        sys.exit(3)
    return chain


def gpu_signed_rounds(lib_tbls, first, n, x):
    """Fallback when no chain file is present: rounds first..first+n-1 whose prev_sig is a per-round
    pseudo-random 96 B string (not the previous signature), signed on the GPU.  Same per-round work."""
    import hashlib

    prev = np.frombuffer(b"".join(hashlib.sha256(b"prev/%d" % r).digest() * 3 for r in range(first, first + n)),
                         np.uint8).reshape(n, 96)
    rr = np.arange(first, first + n, dtype=np.uint64)
    msgs = lib_tbls.beacon_messages(rr - 1, rr, [bytes(p) for p in prev])
    sigs = lib_tbls.sign_batch([x] * n, msgs)
    return prev, sigs


def roofline_of(kt, kernel_units, peak, extra=None, config="head"):
    """Roofline object of the dominant kernel of a timing table {name: (avg us, launches)}: the kernel with
    the largest total time among those profiles/opcounts.json prices; kernel_units[name] = the units all its
    timed launches processed together (per launch: that / launches)."""
    oc = json.load(open(os.path.join(ROOT, "profiles", "opcounts.json")))["per_unit"]
    cands = [(us * n, name, us) for name, (us, n) in kt.items()
             if name in kernel_units and (name in oc or isinstance(kernel_units[name], dict))]
    if not cands:
        return None
    _, name, us = max(cands)
    u = kernel_units[name]
    if isinstance(u, dict):  # a mix of unit kinds {opcounts key: units}: MACs per unit averaged over the mix
        total = sum(u.values())
        macs = sum(c * oc[k]["macs"] for k, c in u.items()) / max(total, 1)
        vmad = sum(c * oc[k].get("vmad", 0) for k, c in u.items()) / max(total, 1)
        units = total / kt[name][1]
    else:
        macs = oc[name]["macs"]
        vmad = oc[name].get("vmad", 0)
        units = u / kt[name][1]
    achieved = macs * units / (us * 1e-6) / 1e12
    issued = vmad * units / (us * 1e-6) / 1e12
    # a rank without a measured peak still reports what it achieved (frac null), never a TypeError
    pk = peak.get("tmac_s") if peak else None
    out = {"bound": "valu-int", "achieved": achieved, "peak": pk, "unit": "TMAC/s",
           "frac": achieved / pk if pk else None, "traffic": traffic_of(name, config), "kernel": name,
           "kernel_avg_us": us, "units_per_launch": units, "macs_per_unit": macs,
           "vmad_per_unit": vmad, "issue_frac": issued / pk if pk else None,
           "peak_source": peak.get("source") if peak else None}
    if extra:
        out.update(extra)
    return out


def pipeline_roofline(kt, checks, rounds, peak, extra=None, config="c5"):
    """Roofline of Recover's per-item pass as the pairing-check pipeline (checks.h): the algorithmic multiply-adds of
    every check the pass ran (profiles/opcounts.json: k_ck_prep[m] by member count m, the same rest per check) and of
    the per-round lines, over the summed HIP-event time of every k_ck_* launch of the call.  None when the call ran
    no k_ck_* kernel."""
    ck = {k: v for k, v in kt.items() if k.startswith("k_ck_")}
    if not ck:
        return None
    oc = json.load(open(os.path.join(ROOT, "profiles", "opcounts.json")))["per_unit"]
    rest = sum(oc[k]["macs"] for k in CK_REST)
    n = sum(checks.values())
    macs = sum(c * (oc["k_ck_prep[%d]" % m]["macs"] + rest) for m, c in checks.items()) + \
        rounds * oc["k_ck_round_lines (per round)"]["macs"]
    us = sum(a * l for a, l in ck.values())
    achieved = macs / (us * 1e-6) / 1e12
    pk = peak.get("tmac_s") if peak else None
    trf = traffic_of("k_ck_* pipeline", config)
    out = {"bound": "valu-int", "achieved": achieved, "peak": pk, "unit": "TMAC/s", "frac": achieved / pk if pk else None,
           "traffic": trf, "kernel": "k_ck_* pipeline", "kernel_avg_us": us, "units_per_launch": n,
           "macs_per_unit": macs / max(n, 1), "issue_frac": None, "peak_source": peak.get("source") if peak else None,
           "per_kernel_share": {k: round(a * l / us, 4) for k, (a, l) in ck.items()}}
    if extra:
        out.update(extra)
    return out


# the per-check kernels of the pipeline after the members' sums (profiles/opcounts.json keys)
CK_REST = ("k_ck_lines2", "k_ck_miller", "k_ck_easy", "k_ck_expsq (5 per check)", "k_ck_expdec (5 per check)",
           "k_ck_final")


def xr_roofline(kt, counts, quads, peak, extra=None):
    """Roofline of the cross-round isolation of failed single-key batches (xr.h) as a whole: the algorithmic
    multiply-adds of its quad sums (2 sides per quad) and of the checks of each level (counts: dg_isolation_counts
    deltas; level 1 groups of 4 quads, level 2 quads, level 3 single rounds; each check h_eff + lines of its hash side
    and the pipeline's per-check rest), over the summed HIP-event time of every k_xg_* / k_xq_* / k_ck_* launch."""
    ks = {k: v for k, v in kt.items() if k.startswith(("k_ck_", "k_xg_", "k_xq_"))}
    if not ks or not sum(counts):
        return None
    oc = json.load(open(os.path.join(ROOT, "profiles", "opcounts.json")))["per_unit"]
    per_check = oc["k_xg_hlines"]["macs"] + sum(oc[k]["macs"] for k in CK_REST)
    macs = (2 * quads * oc["k_xq_sum (per quad side)"]["macs"] + counts[0] * (oc["k_xg_prep[level 1, 4 quads]"]["macs"] +
            per_check) + counts[1] * (oc["k_xg_prep[level 2]"]["macs"] + per_check) + counts[2] * per_check)
    us = sum(a * l for a, l in ks.values())
    achieved = macs / (us * 1e-6) / 1e12
    pk = peak.get("tmac_s") if peak else None
    out = {"bound": "valu-int", "achieved": achieved, "peak": pk, "unit": "TMAC/s", "frac": achieved / pk if pk else None,
           "traffic": traffic_of("xr pipeline", "c2neg"), "kernel": "xr isolation (k_xq/k_xg/k_ck_*)",
           "kernel_avg_us": us, "units_per_launch": sum(counts), "macs_per_unit": macs / max(sum(counts), 1),
           "issue_frac": None, "checks_by_level": list(counts), "quads": quads,
           "per_kernel_share": {k: round(a * l / us, 4) for k, (a, l) in ks.items()}}
    if extra:
        out.update(extra)
    return out


COMPACT_ROOF = ("bound", "achieved", "peak", "unit", "frac", "traffic", "kernel", "kernel_avg_us", "units_per_launch",
                "macs_per_unit", "issue_frac", "chip", "overlapped")


def compact_roofline(r):
    """The roofline fields the printed line keeps (the rest goes to the side file)."""
    if not r:
        return r
    out = {k: r[k] for k in COMPACT_ROOF if k in r}
    for k in ("chip", "overlapped"):
        if isinstance(out.get(k), dict):
            out[k] = {q: v for q, v in out[k].items() if q != "note"}
    return out


# ------------------------------------------------------------------------------------------ CPU baselines
def cpu_verify(pk, msgs, sigs, threads, seconds=8.0):
    """C2 on the host: the CPU twin (C port of the reference algorithm: one full pairing check per beacon)
    on a bounded sample of the same rounds."""
    from oracle import twin

    n0 = 32
    t0 = time.time()
    twin.verify_batch(pk, msgs[:n0], sigs[:n0], threads=1)
    per = (time.time() - t0) / n0
    n = int(min(len(sigs), max(n0, seconds * threads / per)))
    t0 = time.time()
    st = twin.verify_batch(pk, msgs[:n], sigs[:n], threads=threads)
    dt = time.time() - t0
    assert not st.any(), "CPU twin rejected a valid round"
    return {"value": n / dt, "unit": "rounds/s", "cores": threads, "kind": "port",
            "sample": "%d rounds of the same chain, CPU twin (oracle/twin, C restatement of the kyber per-item "
                      "bls.Verify: 2 Miller loops + final exp per round), %d threads, %.1f s" % (n, threads, dt)}


def cpu_c1(threads, rounds=1000):
    """BASELINE configs[0] (C1) on the host: n = 5, t = 3; per round 5 tbls.Sign, Recover (re-verifying each
    examined share) and VerifyRecovered (beacon/beacon_test.go:41-93, beacon/beacon.go:433-494)."""
    from oracle import twin

    g = json.load(open(os.path.join(ROOT, "tests", "golden", "groups.json")))["t3"]
    coeffs = S.poly_coeffs(3)
    shares = [S.share_value(coeffs, i) for i in range(5)]
    commits = [bytes.fromhex(c) for c in g]
    import hashlib

    msgs = np.frombuffer(b"".join(hashlib.sha256(b"c1/%d" % r).digest() for r in range(rounds)),
                         np.uint8).reshape(rounds, 32)
    t0 = time.time()
    _, ok = twin.c1_batch(commits, 3, 5, shares, msgs, threads=threads)
    dt = time.time() - t0
    assert ok == rounds, "CPU twin C1 round failed"
    return {"value": rounds / dt, "unit": "rounds/s", "cores": threads, "kind": "port",
            "sample": "%d rounds, n=5 t=3: 5 Signs + Recover + VerifyRecovered per round, CPU twin, %d threads, "
                      "%.1f s" % (rounds, threads, dt)}


def cpu_recover(commits, t, n, msgs, parts, threads, seconds=8.0, label=""):
    """Recover (the kyber algorithm: VerifyPartial of each examined share in input order, Lagrange over the
    first t valid) on the host over a bounded sample of the same rounds."""
    from oracle import twin

    t0 = time.time()
    twin.recover_batch(commits, t, n, msgs[:1], parts[:1], threads=1)
    per = time.time() - t0
    R = int(min(len(msgs), max(threads, seconds * threads / per)))
    t0 = time.time()
    _, rs, ss = twin.recover_batch(commits, t, n, msgs[:R], parts[:R], threads=threads)
    dt = time.time() - t0
    return {"value": R / dt, "unit": "recovers/s", "cores": threads, "kind": "port",
            "statuses_per_s": int((ss != 255).sum()) / dt,
            "sample": "%d rounds of the same %s partials, CPU twin tbls.Recover, %d threads, %.1f s"
                      % (R, label, threads, dt)}, (rs, ss, R)


def cpu_verify_partials(commits, msgs, parts, threads, seconds=6.0):
    """VerifyPartial (beacon/beacon.go:148: PubPoly.Eval of the share's index + bls.Verify) on the host, one CPU-twin
    call per partial, `threads` at once (ctypes releases the GIL), over a bounded sample of the same partials ->
    partials/s."""
    from concurrent.futures import ThreadPoolExecutor

    from oracle import twin

    R, n = parts.shape[0], parts.shape[1]
    items = [(r, j) for r in range(R) for j in range(n)]
    t0 = time.time()
    twin.verify_partial(commits, bytes(msgs[0]), bytes(parts[0, 0]))
    per = time.time() - t0
    m = int(min(len(items), max(threads, seconds * threads / max(per, 1e-6))))
    t0 = time.time()
    with ThreadPoolExecutor(threads) as ex:
        st = list(ex.map(lambda it: twin.verify_partial(commits, bytes(msgs[it[0]]), bytes(parts[it[0], it[1]])),
                         items[:m]))
    dt = time.time() - t0
    assert not any(st), "CPU twin rejected a valid partial"
    return m / dt, "%d partials (first %d rounds x %d), CPU twin VerifyPartial, %d threads, %.1f s" % (
        m, -(-m // n), n, threads, dt)


class RoundSource:
    """Rounds 1..total with their prev_sig and signature for the Recover lines: the linked chain file when one
    holds them, else GPU-signed rounds whose prev_sig is pseudo-random (gpu_signed_rounds: the same per-round
    work; only the syncFrom line needs the links and is skipped then)."""

    def __init__(self, tbls, total, allow_unlinked=False):
        chain = require_chain(total, allow_unlinked)
        self.linked = chain is not None
        if self.linked:
            self.sigs = chain
        else:
            self.prevs, self.sigs = gpu_signed_rounds(tbls, 1, total, S.master_secret())

    def prev(self, r):
        """prev_sig of round r (1-based)"""
        if self.linked:
            return bytes(self.sigs[r - 2]) if r >= 2 else S.GENESIS_SEED
        return bytes(self.prevs[r - 1])


# --------------------------------------------------------------------------------------- Recover lines
def make_group_rounds(tbls, src, first, R, t, n):
    """Partials sigma_{i,r} = x_i H(m_r) of an (n, t) group for chain rounds first..first+R-1, signed on the
    GPU (untimed).  Returns (pub, commits, shares, msgs (R, 32), parts (R, n, 98))."""
    g = json.load(open(os.path.join(ROOT, "tests", "golden", "groups.json")))["t%d" % t]
    commits = [bytes.fromhex(c) for c in g]
    pub = tbls.PubPoly(commits)
    coeffs = S.poly_coeffs(t)
    shares = [S.share_value(coeffs, i) for i in range(n)]
    rounds = np.arange(first, first + R, dtype=np.uint64)
    prev = [src.prev(r) for r in rounds.tolist()]
    msgs = tbls.beacon_messages(rounds - 1, rounds, prev)
    parts = np.empty((R, n, 98), np.uint8)
    step = max(1, 2000000 // n)
    for a in range(0, R, step):
        b = min(R, a + step)
        sc = [shares[i] for _ in range(a, b) for i in range(n)]
        idx = [i for _ in range(a, b) for i in range(n)]
        parts[a:b] = tbls.sign_batch(sc, np.repeat(msgs[a:b], n, axis=0), idx).reshape(b - a, n, 98)
    return pub, commits, shares, msgs, parts


def gather_recover(sigs, rs, ss, world, total):
    """All-gather of the Recover outputs of every rank's contiguous range (RCCL; device tensors from
    dg_recover_dev go in as they are) -> numpy (total, ...)."""
    import torch

    from drand_amd import shard

    dev = torch.device("cuda", torch.cuda.current_device())
    xs = [x if isinstance(x, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(x)).to(dev) for x in (sigs, rs, ss)]
    if world > 1:
        xs = [shard.allgather_rows(x, world, total) for x in xs]
    out = [x.cpu().numpy() for x in xs]
    return out[0], out[1].reshape(-1), out[2]


def timed_ranks(fn, world):
    """fn() between barriers; the max over ranks of its wall time."""
    import torch
    import torch.distributed as dist

    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    res = fn()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64, device=torch.device("cuda", torch.cuda.current_device()))
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    return res, dt


def recover_bench(L, tbls, shard, src, R_total, t, n, world, rank, peak, steps=2):
    """BASELINE configs[2]: kyber's tbls.Recover for an (n, t) group -- VerifyPartial of the partials
    in input order up to the t-th valid one, Lagrange interpolation -- over R_total rounds of the chain, each rank its contiguous range through dg_recover_dev with the messages and
    98 B partials already resident in HBM (the headline `value`, like the verify headline), then the RCCL
    all-gather of the recovered signatures, round statuses and share statuses.  `host_api_value` is the same
    work through the host-buffer dg_recover (the partials cross PCIe inside the call); round-1 numbers were
    host-buffer rates, so compare host_api_value with them.  Every recovered signature must equal the
    chain's byte for byte."""
    a, b = shard.round_range(R_total, world, rank)
    R = b - a
    t0 = time.perf_counter()
    import torch

    pub, commits, shares, msgs, parts = make_group_rounds(tbls, src, a + 1, R, t, n)
    gen_s = time.perf_counter() - t0
    dev = torch.device("cuda", torch.cuda.current_device())
    d_msgs = torch.from_numpy(np.ascontiguousarray(msgs)).to(dev)
    d_parts = torch.from_numpy(np.ascontiguousarray(parts)).to(dev)
    tbls.recover_batch_dev(pub, d_msgs, d_parts, t, n, seed=5)  # warmup (workspace growth)
    dts = []
    for s in range(steps):
        (sigs, rs, ss), dt = timed_ranks(lambda: tbls.recover_batch_dev(pub, d_msgs, d_parts, t, n, seed=6 + s), world)
        dts.append(dt)
    (gs, grs, gss), gdt = timed_ranks(lambda: gather_recover(sigs, rs, ss, world, R_total), world)
    assert not grs.any() and np.array_equal(gs, src.sigs[:R_total]), "recovered signatures differ from the chain"
    assert (gss[:, :t] == 0).all() and (gss[:, t:] == 255).all(), "share statuses"
    dt = min(dts)
    # BASELINE configs[2] as written: VerifyPartial of EVERY partial (ProcessBeacon, beacon/beacon.go:148: all n of
    # every round) + Recover (:488).  Timed as dg_verify_partials_dev over all R x n partials, then (a) kyber's
    # Recover, which re-verifies the examined prefix (the dg_recover_dev time above), and (b) the Lagrange half
    # from those verdicts (dg_recover_verified_dev).
    tbls.verify_partial_batch_dev(pub, d_msgs, d_parts, seed=3)  # warmup (workspace growth at R x n items)
    vdts = []
    for s in range(steps):
        d_vst, vdt = timed_ranks(lambda: tbls.verify_partial_batch_dev(pub, d_msgs, d_parts, seed=30 + s), world)
        vdts.append(vdt)
    vdt = min(vdts)
    assert int(d_vst.max().item()) == 0, "VerifyPartial rejected a valid partial"
    tbls.recover_verified_batch_dev(d_parts, d_vst, t, n)  # warmup
    (vs, vrs, vss), rvdt = timed_ranks(lambda: tbls.recover_verified_batch_dev(d_parts, d_vst, t, n), world)
    assert not int(vrs.max().item()) and torch.equal(vs, sigs), "Recover from the verdicts differs"
    L.check(L.lib().dg_set_timing(1))
    tbls.verify_partial_batch_dev(pub, d_msgs, d_parts, seed=8)
    vkt = L.timings()
    L.check(L.lib().dg_set_timing(0))
    vroof = roofline_of(vkt, {"k_exp_pm3d4": 4 * R + 2 * R * n, "k_dec_p1": R * n, "k_dec_p2": R * n,
                              "k_dec_p3": R * n}, peak, {"timing": "HIP events on the launch stream, one call"}, "c3vp")
    vp_line = {"metric": "BASELINE configs[2]: VerifyPartial on all %d shares of every round + Lagrange Recover, n=%d "
                         "t=%d (recovers/s)" % (n, n, t),
               "value": R_total / (vdt + dt + gdt), "unit": "recovers/s",
               "value_recover_from_verdicts": R_total / (vdt + rvdt + gdt),
               "partials_verified_per_s": R_total * n / vdt, "verify_partials_s": vdt, "recover_s": dt,
               "recover_from_verdicts_s": rvdt, "roofline": vroof,
               "kernel_avg_us": {k_: round(v[0], 1) for k_, v in vkt.items()},
               "note": "value: dg_verify_partials_dev over all R x n partials (HBM-resident) + kyber Recover "
                       "(dg_recover_dev, which re-verifies its examined prefix); value_recover_from_verdicts: the "
                       "same VerifyPartial pass + dg_recover_verified_dev (Lagrange from the verdicts, no second "
                       "pairing); every status OK and every signature equal to the chain's"}
    del d_vst
    # the host-buffer entry point (dg_recover): the 98 B partials cross PCIe inside the call
    (hs, hrs, hss), host_dt = timed_ranks(lambda: tbls.recover_batch(pub, msgs, parts, t, n, seed=7), world)
    assert np.array_equal(hs, gs[a:b]) and np.array_equal(hss, gss[a:b]), "host and device Recover differ"
    # per-kernel timing of one more call: the dominant kernel's roofline
    L.check(L.lib().dg_set_timing(1))
    tbls.recover_batch_dev(pub, d_msgs, d_parts, t, n, seed=9)
    kt = L.timings()
    L.check(L.lib().dg_set_timing(0))
    # k_rc_straus: one unit = one round (its four psi-component lanes), priced at the C3 index set 0..32
    # (every round valid: the batch covers each round's first t partials, the window; the rest are not decoded)
    units = {"k_decode_items": R * t, "k_rc_straus": R, "k_h2c_uncleared": R,
             "k_exp_pm3d4": 4 * R + 2 * R * t, "k_dec_p1": R * t, "k_dec_p2": R * t, "k_dec_p3": R * t}
    roof = roofline_of(kt, units, peak, {"timing": "HIP events on the launch stream, one dg_recover call"}, "c3")
    out = {"metric": "Recover/s at n=%d t=%d (kyber tbls.Recover: partials VerifyPartial'd in input order up to the "
                     "t-th valid, Lagrange-interpolated)" % (n, t),
           "value": R_total / (dt + gdt), "unit": "recovers/s", "n_gpus": world, "rounds": R_total,
           "rounds_per_gpu": R, "partials_per_round": n, "s_per_step": dt, "allgather_s": gdt,
           "partials_examined_per_s": int((gss != 255).sum()) / (dt + gdt), "partials_generated_s": gen_s,
           "host_api_s_per_step": host_dt, "host_api_value": R_total / (host_dt + gdt),
           "roofline": roof, "kernel_avg_us": {k: round(v[0], 1) for k, v in kt.items()},
           "kernel_launches": {k: v[1] for k, v in kt.items()},
           "note": "inputs resident in HBM (dg_recover_dev), outputs all-gathered (RCCL) and equal to the chain's "
                   "signatures; host_api_value: the host-buffer dg_recover, with the PCIe transfer of %d MB of "
                   "partials per GPU inside the call" % (R * n * 98 // 10**6)}
    return out, (commits, msgs, parts), vp_line


def make_c5_inputs(tbls, shard, src, R_total, world, rank, t=129, n=256, frac=0.10, n_short=3):
    """configs[4]'s inputs for this rank's contiguous range of R_total rounds: n partials per round signed by the
    GPU (dg_sign), ~frac of the (round, share) cells corrupted with the six modes of tools/corrupt.py (pattern of the
    GLOBAL round numbers), `n_short` rounds with too few valid shares.  Returns (pub, commits, msgs, parts, bad, short,
    items, gen_s, a, b)."""
    from tools import corrupt

    g = json.load(open(os.path.join(ROOT, "tests", "golden", "groups.json")))["t%d" % t]
    commits = [bytes.fromhex(c) for c in g]
    pub = tbls.PubPoly(commits)
    coeffs = S.poly_coeffs(t)
    shares = [S.share_value(coeffs, i) for i in range(n)]
    a, b = shard.round_range(R_total, world, rank)
    R = b - a
    rounds = np.arange(a + 1, b + 2, dtype=np.uint64)  # one extra round for the "other_round" mode
    prev = [src.prev(r) for r in rounds.tolist()]
    msgs_all = tbls.beacon_messages(rounds - 1, rounds, prev)
    msgs = msgs_all[:R]
    t0 = time.perf_counter()
    parts = tbls.sign_batch([shares[i] for _ in range(R) for i in range(n)], np.repeat(msgs, n, axis=0),
                            [i for _ in range(R) for i in range(n)]).reshape(R, n, 98)
    # corruption pattern of the GLOBAL round numbers, so it does not depend on the rank count
    items = [it for it in corrupt.pick(R_total, n, frac) if a <= it[0] < b]
    items = [(r - a, j, m) for r, j, m in items]
    short = set(r - a for r in range(n_short) if a <= r < b)
    items = [it for it in items if it[0] not in short] + [(r, j, "random_bytes") for r in sorted(short)
                                                           for j in range(n - t + 2)]

    def resign(reqs):
        sc = [shares[idx] + ds for _, idx, ds, _ in reqs]
        return tbls.sign_batch(sc, np.stack([msgs_all[r + dr] for r, _, _, dr in reqs]))

    corrupt.corrupt_batch(parts, items, n, resign)
    gen_s = time.perf_counter() - t0
    bad = np.zeros((R, n), dtype=bool)
    for r, j, _ in items:
        bad[r, j] = True
    return pub, commits, msgs, parts, bad, short, items, gen_s, a, b


def adversarial_bench(L, tbls, shard, src, R_total, world, rank, peak, t=129, n=256, frac=0.10, n_short=3, vp_neg=True):
    """BASELINE configs[4]: n = 256, t = 129, ~10% of the (round, share) cells corrupted with the six
    cycling modes of tools/corrupt.py, plus `n_short` rounds with more than n - t corrupted shares (-> "not
    enough shares"); each rank its contiguous range of R_total rounds through dg_recover_dev (inputs resident
    in HBM; the batch equation fails, so the examined prefix of every round takes the per-item pass: group
    tests of up to 4 shares -- a passed group's members are accepted with error probability <= 2^-63 (odd 64-bit weights) -- and
    single pairing checks for the members of failed groups; DG_GROUP=1 makes every check a single one), then
    the all-gather of the outputs.  Checked without the CPU: recovered signatures equal the chain's, exactly the short rounds
    report NOT_ENOUGH, every examined corrupted share is rejected and every examined clean one accepted
    (per-share parity with the CPU twin is tests/test_gpu_parity.py's job)."""
    pub, commits, msgs, parts, bad, short, items, gen_s, a, b = make_c5_inputs(tbls, shard, src, R_total, world, rank,
                                                                             t, n, frac, n_short)
    R = b - a
    import torch

    dev = torch.device("cuda", torch.cuda.current_device())
    d_msgs = torch.from_numpy(np.ascontiguousarray(msgs)).to(dev)
    d_parts = torch.from_numpy(np.ascontiguousarray(parts)).to(dev)
    tbls.recover_batch_dev(pub, d_msgs, d_parts, t, n, seed=11)  # warmup
    (d_sigs, d_rs, d_ss), dt = timed_ranks(lambda: tbls.recover_batch_dev(pub, d_msgs, d_parts, t, n, seed=12), world)
    sigs, rs, ss = (x.cpu().numpy() for x in (d_sigs, d_rs, d_ss))
    (hs, hrs, hss), host_dt = timed_ranks(lambda: tbls.recover_batch(pub, msgs, parts, t, n, seed=12), world)
    assert np.array_equal(hs, sigs) and np.array_equal(hrs, rs) and np.array_equal(hss, ss), "host / device differ"
    ok_r = np.array([r not in short for r in range(R)], dtype=bool)
    assert np.array_equal(rs != 0, ~ok_r) and (rs[~ok_r] == 5).all(), "round statuses"
    assert np.array_equal(sigs[ok_r], src.sigs[a:b][ok_r]), "recovered signatures differ from the chain"
    examined = ss != 255
    assert (ss[examined & bad] != 0).all() and (ss[examined & ~bad] == 0).all(), "share statuses"
    (gs, grs, gss), gdt = timed_ranks(lambda: gather_recover(d_sigs, d_rs, d_ss, world, R_total), world)
    assert gs.shape == (R_total, 96) and gss.shape == (R_total, n)
    L.check(L.lib().dg_set_timing(1))
    g0 = L.group_counts()
    tbls.recover_batch_dev(pub, d_msgs, d_parts, t, n, seed=13)
    kt = L.timings()
    g1 = L.group_counts()
    L.check(L.lib().dg_set_timing(0))
    checks = {"k_ck_prep[%d]" % (m + 1): g1[m] - g0[m] for m in range(4)}
    # the per-item pass as a whole (the pairing-check pipeline of checks.h); k_rs_sac: one unit = one round's joint
    # column MSM (priced at t = 129 over a scattered index set)
    ext = {"timing": "HIP events on the launch stream, one dg_recover call", "checks_by_members": checks}
    roof = pipeline_roofline(kt, {m + 1: g1[m] - g0[m] for m in range(4)}, R, peak, ext, "c5")
    rs_roof = roofline_of({k: v for k, v in kt.items() if k == "k_rs_sac"}, {"k_rs_sac": R}, peak, None, "c5")
    vpn = vp_negative_bench(L, tbls, pub, d_msgs, d_parts, bad, world, peak) if vp_neg else None
    ncorrupt = np.array([len(items)], np.int64)
    if world > 1:
        import torch
        import torch.distributed as dist

        c = torch.from_numpy(ncorrupt).cuda()
        dist.all_reduce(c)
        ncorrupt = c.cpu().numpy()
    return {"metric": "adversarial Recover/s at n=%d t=%d, %.0f%% of shares corrupted (C5)" % (n, t, 100 * frac),
            "value": R_total / (dt + gdt), "unit": "recovers/s", "n_gpus": world, "rounds": R_total,
            "rounds_per_gpu": R, "partials_per_round": n, "corrupted_shares": int(ncorrupt[0]),
            "short_rounds": n_short, "s_per_step": dt, "allgather_s": gdt,
            "statuses_per_s": int((gss != 255).sum()) / (dt + gdt), "setup_s": gen_s, "roofline": roof,
            "rs_sac_roofline": rs_roof,
            "host_api_s_per_step": host_dt, "host_api_value": R_total / (host_dt + gdt),
            "kernel_avg_us": {k: round(v[0], 1) for k, v in kt.items()},
            "kernel_launches": {k: v[1] for k, v in kt.items()},
            "note": "inputs resident in HBM (dg_recover_dev); the batch equation fails, so the examined prefix of "
                    "every round takes the per-item pass (group tests, then single checks); outputs all-gathered "
                    "(RCCL); host_api_value: the host-buffer dg_recover with the PCIe transfer of %d MB of partials "
                    "per GPU inside the call" % (R * n * 98 // 10**6)}, (commits, msgs, parts,
                                                                                             ss, rs), vpn


def c1_gpu(L, tbls, reps=3, rounds=1000):
    """BASELINE configs[0] (C1) on the GPU, the same work as cpu_c1: 5 tbls.Sign per round (dg_sign), Recover
    (dg_recover: VerifyPartial of the shares + Lagrange) and VerifyRecovered (dg_verify) of 1000 rounds."""
    import hashlib

    g = json.load(open(os.path.join(ROOT, "tests", "golden", "groups.json")))["t3"]
    pub = tbls.PubPoly([bytes.fromhex(c) for c in g])
    coeffs = S.poly_coeffs(3)
    shares = [S.share_value(coeffs, i) for i in range(5)]
    msgs = np.frombuffer(b"".join(hashlib.sha256(b"c1/%d" % r).digest() for r in range(rounds)),
                         np.uint8).reshape(rounds, 32)

    def run():
        parts = tbls.sign_batch([shares[i] for _ in range(rounds) for i in range(5)], np.repeat(msgs, 5, axis=0),
                                [i for _ in range(rounds) for i in range(5)]).reshape(rounds, 5, 98)
        sigs, rs, _ = tbls.recover_batch(pub, msgs, parts, 3, 5)
        st = tbls.verify_recovered_batch(pub.commit(), msgs, sigs)
        assert not rs.any() and not st.any()
        return sigs

    run()
    t0 = time.perf_counter()
    for _ in range(reps):
        run()
    dt = (time.perf_counter() - t0) / reps
    return {"metric": "C1: n=5 t=3, 5 Signs + Recover + VerifyRecovered per round (BASELINE configs[0])",
            "value": rounds / dt, "unit": "rounds/s", "rounds": rounds, "s_per_step": dt,
            "note": "three blocking host-buffer calls per 1000 rounds (dg_sign, dg_recover, dg_verify)"}


def live_latency(L, tbls, commits, msgs, parts, t, n, reps=20):
    """SURVEY §8(f) row 4, the live round (beacon/beacon.go:472-494): one round's Recover with the
    VerifyPartial verdicts ProcessBeacon already holds (dg_recover_verified: no re-verification) and the
    VerifyRecovered of its output, per call; plus the full dg_recover of one round for comparison."""
    pub = tbls.PubPoly(commits)
    m1, p1 = msgs[:1], parts[:1]
    st = np.zeros((1, n), np.uint8)
    sig, rs, _ = tbls.recover_verified_batch(pub, m1, p1, st, t, n)
    assert not rs.any()
    out = {}
    for name, fn in (("recover_verified_ms", lambda: tbls.recover_verified_batch(pub, m1, p1, st, t, n)),
                     ("recover_full_ms", lambda: tbls.recover_batch(pub, m1, p1, t, n)),
                     ("verify_recovered_ms", lambda: tbls.verify_recovered_batch(pub.commit(), m1, sig))):
        fn()
        t0 = time.perf_counter()
        for _ in range(reps):
            fn()
        out[name] = (time.perf_counter() - t0) / reps * 1e3
    out.update({"metric": "live-round latency, one round at n=%d t=%d (ms per call)" % (n, t),
                "note": "host-buffer blocking calls; recover_verified takes the ProcessBeacon verdicts "
                        "(beacon/beacon.go:148) instead of re-verifying the shares (:488)"})
    return out


def sync_bench(chain_sigs, R, batch=25000):
    """syncFrom catch-up (drand_amd/bulk.sync_from) of R linked chain rounds from the
    genesis seed, as Beacon objects streamed by one peer, `batch` rounds per GPU call (links + one RLC
    multi-pairing per batch); host objects, PCIe and the per-batch blocking calls inside the timed
    region.  Every round must be stored."""
    from drand_amd import bulk

    pk = S.GROUP_PK
    bs = [bulk.Beacon(r - 1, S.GENESIS_SEED if r == 1 else bytes(chain_sigs[r - 2]), r, bytes(chain_sigs[r - 1]))
          for r in range(1, R + 1)]
    got = []
    t0 = time.perf_counter()
    res = bulk.sync_from(pk, 0, S.GENESIS_SEED, [bs], put=got.append, batch=batch)
    dt = time.perf_counter() - t0
    assert res.stored == R and got[-1].round == R, "sync_from did not store the whole chain"
    return {"metric": "syncFrom catch-up rounds/s (bulk.sync_from, beacon/beacon.go:529-607)", "value": R / dt,
            "unit": "rounds/s", "rounds": R, "batch": batch, "s": dt,
            "note": "host Beacon objects -> dg_check_links + dg_verify_beacons per batch (host-buffer API, blocking)"}


MAX_BATCH = 524288  # rounds per device batch by default at most (~6 GB of workspace per set at this size)


def batch_bounds(n, batch=0):
    """The device batches of a rank's n rounds: [(lo, hi)], contiguous and balanced.  batch = 0 (default): one batch
    when n <= MAX_BATCH -- at N = 8 the 1M chain gives every rank 125k rounds, so each rank runs the N = 1 step (one
    batch, its verdicts packed and all-gathered on the batch's own stream) instead of two batches and a side stream;
    at N = 2 and 4 (500k, 250k rounds) one batch as well."""
    cap = batch if batch > 0 else MAX_BATCH
    nb = max(1, -(-n // cap))
    return [(n * i // nb, n * (i + 1) // nb) for i in range(nb)]


def consume_on_batch_stream(nbatches, use_sync=False):
    """Whether a step's consumers (the bitmap pack and its RCCL all-gather) go on the batch's own stream
    (dg_last_batch_stream) -- no cross-stream wait at all, which with HIP's default 4 hardware queues stalls whatever
    shares the waiting queue -- at every world size when the rank's step is one asynchronous batch;
    several batches (or the blocking entry point) need a side stream that waits for them all."""
    return nbatches == 1 and not use_sync


def negative_positions(G):
    """Global 0-based positions of the corrupted rounds of the negative lines: 1% of G, the deterministic positions
    of tests/test_gpu_round2.py::test_sharded_1m_chain_equals_one_batch."""
    return np.unique((np.arange(G // 100, dtype=np.int64) * 7919 + 13) % G)


def negative_bench(L, args, step, drain, sig_src, d_sts, nbuf, counter, n, a, G, world, peak, bounds):
    """BASELINE configs[1] with SURVEY §8(d) C2's negative variant: the same overlapped, HBM-resident steps as the
    headline, but 1% of the signatures replaced (at negative_positions) by the valid signature of the next round, so
    every batch equation fails and each batch isolates its bad rounds (beacon/chain.go:65-71: kyber's verdict is per
    beacon).  Every step's verdicts must flag exactly the replaced rounds (status 1, bad signature)."""
    import torch

    from drand_amd import shard

    d_sig = sig_src[0]
    bad = negative_positions(G)
    loc = bad[(bad >= a) & (bad < a + n)] - a
    neg = d_sig.clone()
    src = torch.from_numpy(np.where(loc + 1 < n, loc + 1, loc - 1)).to(d_sig.device)
    neg[torch.from_numpy(loc).to(d_sig.device)] = d_sig[src]
    want = torch.zeros(n, dtype=torch.uint8, device=d_sig.device)
    want[torch.from_numpy(loc).to(d_sig.device)] = L.ST_BAD_SIG
    sig_src[0] = neg
    try:
        for w in range(max(1, args.warmup)):
            step(2000 + w)
        drain()
        fb0 = L.fallback_count()
        if world > 1:
            import torch.distributed as dist

            dist.barrier()
        c0 = counter[0]
        t0 = time.perf_counter()
        bits = [step(3000 + s) for s in range(args.neg_steps)]
        drain()
        if world > 1:
            dist.barrier()
        dt = max_over_ranks(time.perf_counter() - t0, world)
        for i in sorted(set(c % nbuf for c in range(max(c0, counter[0] - nbuf), counter[0]))):
            assert torch.equal(d_sts[i], want), "c2_negative: verdicts differ from the replaced rounds"
        want_bits = shard.allgather_verdicts(want, world, m=(max(y - x for x, y in (shard.round_range(G, world, q)
                                                                                    for q in range(world))) + 7) // 8)
        assert all(torch.equal(b_, want_bits) for b_ in bits), "c2_negative: gathered bitmap"
        fallbacks = L.fallback_count() - fb0
        L.check(L.lib().dg_set_timing(1))
        x0 = L.isolation_counts()
        [step(3000 + s) for s in range(args.neg_steps)]
        drain()
        kt = L.timings()
        x1 = L.isolation_counts()
        L.check(L.lib().dg_set_timing(0))
    finally:
        sig_src[0] = d_sig
    counts = [b_ - a_ for a_, b_ in zip(x0, x1)]
    nb = len(bounds)
    quads = sum((hi - lo + 3) // 4 for lo, hi in bounds) * args.neg_steps
    ext = {"timing": "HIP events, instrumented replay of the timed steps (overlapped)"}
    roof = xr_roofline(kt, counts, quads, peak, ext)
    if roof is None:
        roof = roofline_of(kt, {"k_exp_pm3d4": 6 * n * args.neg_steps}, peak, ext)
    iso = {k: v for k, v in kt.items() if k.startswith(("k_ck_", "k_xg_", "k_xq_"))}
    tot = sum(u * c for u, c in kt.values()) or 1.0
    return {"metric": "configs[1] negative: verified beacon rounds/s, 100k-round chain with 1%% of sigma replaced "
                      "(%d rounds), exact bitmap" % len(bad),
            "value": G * args.neg_steps / dt, "unit": "rounds/s", "steps": args.neg_steps,
            "ms_per_step": dt / args.neg_steps * 1e3, "corrupted_rounds": int(len(bad)), "batch_fallbacks": fallbacks,
            "checks_per_batch": [round(c / max(nb * args.neg_steps, 1), 1) for c in counts],
            "isolation_kernel_share": round(sum(u * c for u, c in iso.values()) / tot, 4), "roofline": roof,
            "kernel_avg_us": {k: round(v[0], 1) for k, v in kt.items()},
            "kernel_launches": {k: v[1] for k, v in kt.items()},
            "note": "same overlapped HBM-resident steps as the headline; every batch equation fails and the batch "
                    "isolates its bad rounds on the device; bitmap asserted exact every step"}


def vp_negative_bench(L, tbls, pub, d_msgs, d_parts, bad, world, peak, steps=2):
    """dg_verify_partials_dev (ProcessBeacon's VerifyPartial, beacon/beacon.go:148, of every partial) on C5's
    corrupted set: n = 256, t = 129, ~10% of the partials corrupted (six modes) plus the short rounds.  The batch
    equation fails, so every partial gets its own verdict by isolation; each must match the corruption map (corrupted:
    rejected, clean: accepted)."""
    import torch

    tbls.verify_partial_batch_dev(pub, d_msgs, d_parts, seed=40)  # warmup
    dts = []
    for s in range(steps):
        d_vst, dt = timed_ranks(lambda: tbls.verify_partial_batch_dev(pub, d_msgs, d_parts, seed=41 + s), world)
        dts.append(dt)
    st = d_vst.cpu().numpy().reshape(bad.shape)
    assert (st[bad] != 0).all() and (st[~bad] == 0).all(), "vp_negative: statuses differ from the corruption map"
    L.check(L.lib().dg_set_timing(1))
    g0 = L.group_counts()
    tbls.verify_partial_batch_dev(pub, d_msgs, d_parts, seed=49)
    kt = L.timings()
    g1 = L.group_counts()
    L.check(L.lib().dg_set_timing(0))
    dt = min(dts)
    R = bad.shape[0]
    roof = pipeline_roofline(kt, {m + 1: g1[m] - g0[m] for m in range(4)}, R, peak,
                             {"timing": "HIP events on the launch stream, one call"}, "c5vp")
    torch.cuda.synchronize()
    return {"metric": "VerifyPartial of all n=256 partials per round, C5's 10%-corrupted set (partials/s)",
            "value": bad.size * world / dt, "unit": "partials/s", "s_per_step": dt, "corrupted": int(bad.sum()),
            "roofline": roof, "kernel_avg_us": {k: round(v[0], 1) for k, v in kt.items()},
            "kernel_launches": {k: v[1] for k, v in kt.items()},
            "note": "HBM-resident partials; batch equation fails; statuses asserted against the corruption map"}


def max_over_ranks(x, world):
    """max of a float over the ranks (the device tensor of the rank's GPU; CPU under gloo)."""
    if world == 1:
        return x
    import torch
    import torch.distributed as dist

    dev = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend() == "nccl" else torch.device("cpu")
    t = torch.tensor([x], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def measure_peak(shard, local, detail=False):
    """The roofline denominator of this rank's GPU: v_mad_u64_u32 lane-MACs/s with distinct carry destinations
    after 2 s of launches, and the clock the chip held (in-kernel s_memtime / s_memrealtime).  With `detail`
    also the other forms (the VCC-shared round-2 probe, the compiler's form, v_mad_u32_u24, v_mul_lo_u32) for
    the side file.  None (and a log line) if the probe library is missing: callers then report frac null."""
    try:
        pk = shard.mad_peak(local)
    except (OSError, RuntimeError) as e:
        log("peak probe unavailable:", e)
        return None
    if detail:
        pk["forms"] = {}
        for kind, name in ((0, "v_mad_u64_u32 vcc"), (2, "v_mad_u64_u32 compiler"), (3, "v_mad_u32_u24"),
                           (4, "v_mul_lo_u32")):
            try:
                pk["forms"][name] = shard.probe_form(local, kind, warm_s=0.5)
            except (OSError, RuntimeError) as e:
                log("probe form", name, "failed:", e)
    return pk


def headline_roofline(kt, kt_iso, per, peak, G, steps, world, dt):
    """Roofline of the headline's dominant kernel (isolated launches of two blocking batches of `per` rounds),
    its overlapped timing, and the whole-chip MAC rate of the timed steps.  Any rank may call it; a rank
    without a peak gets frac null."""
    if not kt_iso:
        return None
    oc = json.load(open(os.path.join(ROOT, "profiles", "opcounts.json")))["per_unit"]
    # units over the two blocking batches: rounds for the fused kernels, exponentiations (4 per round of
    # hash-to-G2, 2 per signature) for k_exp_pm3d4, map items / items for the phases
    nb2 = 2 * per
    units = {"k_h2c_uncleared": nb2, "k_decode_items": nb2, "k_exp_pm3d4": 6 * nb2, "k_h2c_p2": 2 * nb2,
             "k_h2c_p3": 2 * nb2, "k_dec_p1": nb2, "k_dec_p2": nb2, "k_dec_p3": nb2}
    roof = roofline_of(kt_iso, units, peak,
                       {"timing": "HIP events on the launch stream, blocking batches right after the timed "
                                  "region (the kernel alone on the chip)"})
    if not roof:
        return None
    pk = peak.get("tmac_s") if peak else None
    if roof["kernel"] in kt:
        o_us = kt[roof["kernel"]][0]
        a_o = roof["macs_per_unit"] * roof["units_per_launch"] / (o_us * 1e-6) / 1e12
        roof["overlapped"] = {"kernel_avg_us": o_us, "achieved": a_o, "frac": a_o / pk if pk else None,
                              "note": "instrumented replay of the timed region: the launch shares the chip "
                                      "with the other batches in flight"}
    # whole chip: algorithmic multiply-adds of the per-round work (hash, decode, 16 bucket additions of the two
    # MSMs + 10 of the subgroup-check test windows, mixed: signatures and hashes are stored with Z = 1) over the
    # step time; per-batch fixed work not counted
    per_round = (sum(oc[k]["macs"] for k in ("k_h2c_uncleared", "k_decode_items")) +
                 26 * oc["k_msm_chunks[mixed add]"]["macs"])
    if "k_h2c_p1a" in kt_iso:  # the phase kernels (same algorithm, batch inversions)
        per_round = (6 * oc["k_exp_pm3d4"]["macs"] + oc["k_h2c_p1a+p1b"]["macs"] + 2 * oc["k_h2c_p2"]["macs"] +
                     2 * oc["k_h2c_p3"]["macs"] + oc["k_h2c_p4a+p4b"]["macs"] +
                     sum(oc[k]["macs"] for k in ("k_dec_p1", "k_dec_p2", "k_dec_p3")) +
                     26 * oc["k_msm_chunks[mixed add]"]["macs"])
    chip = per_round * G * steps / world / dt / 1e12
    roof["chip"] = {"macs_per_round": per_round, "achieved": chip, "frac": chip / pk if pk else None,
                    "note": "per GPU"}
    return roof


# keys of a sub-line (recover, adversarial, ...) that go to the side file instead of the printed line
SIDE_KEYS = ("kernel_avg_us", "kernel_launches", "kernel_avg_us_isolated", "kernel_time_share", "note", "sample", "partials_generated_s",
             "rs_sac_roofline",
             "setup_s", "checks_by_members", "timing", "allgather_s", "host_api_s_per_step", "rounds_per_gpu",
             "partials_per_round", "recover_s", "recover_from_verdicts_s", "corrupted_rounds", "corrupted",
             "steps", "isolation_kernel_share")


# sub-lines print a short metric name (the full description is in the side file), and only these roofline and
# cpu_baseline fields: the whole line must stay under 4 KB
SHORT_METRIC = {"recover": "configs[2] kyber Recover/s, n=64 t=33 (examined prefix verified)",
                "c2_verify_all": "configs[2] VerifyPartial(all 64) + Recover, recovers/s",
                "adversarial": "configs[4] adversarial Recover/s, n=256 t=129, 10% corrupted",
                "c1": "configs[0] n=5 t=3: 5 Signs + Recover + VerifyRecovered, rounds/s",
                "live_latency": "live round n=64 t=33, ms per call",
                "sync": "syncFrom catch-up rounds/s",
                "c2_negative": "configs[1] with 1% of sigma replaced: rounds/s, exact bitmap",
                "vp_negative": "VerifyPartial on C5's 10%-corrupted set, partials/s"}
SUB_ROOF = ("kernel", "achieved", "peak", "unit", "frac", "traffic", "issue_frac", "kernel_avg_us")
SUB_CPU = ("value", "unit", "cores", "kind", "all_host_cpus_linear_est", "statuses_match_gpu")


def report(rank, world, head, roof, cpu, lines, tables, tables_out):
    """Rank-dependent end of the bench: every rank may pass partial data (a rank off 0 has no CPU baseline and
    the sub-lines it did not run are None); rank 0 prints the one JSON line and writes the side file.  The
    printed line keeps the headline, the compact roofline and cpu_baseline, and for each sub-line its value,
    compact roofline and cpu_baseline; the per-kernel tables, notes and probe details go to `tables_out`."""
    if rank != 0:
        return None
    side = dict(tables)
    out = {"metric": METRIC, "value": head["value"], "unit": "rounds/s", "n_gpus": world, "steps": head["steps"],
           "warmup": head["warmup"], "ms_per_step": head["ms_per_step"], "higher_is_better": True,
           "scaling": head["scaling"], "vs_baseline": None, "dtype": "u32 (381-bit Fp, 12x32-bit limbs)",
           "data": head["data"], "config": head["config"], "roofline": compact_roofline(roof),
           "cpu_baseline": cpu, "batch_fallbacks": head.get("batch_fallbacks")}
    side["roofline"] = roof
    for name, line in lines.items():
        if line is None:
            out[name] = None
            continue
        line = dict(line)
        side[name] = {k: line.pop(k) for k in SIDE_KEYS if k in line}
        if name in SHORT_METRIC and "metric" in line:  # the long description goes to the side file
            side[name]["metric"] = line["metric"]
            line["metric"] = SHORT_METRIC[name]
        if isinstance(line.get("roofline"), dict):
            side[name]["roofline"] = line["roofline"]
            line["roofline"] = {k: v for k, v in compact_roofline(line["roofline"]).items() if k in SUB_ROOF}
        if isinstance(line.get("cpu_baseline"), dict):
            side[name]["cpu_baseline"] = line["cpu_baseline"]
            line["cpu_baseline"] = {k: v for k, v in line["cpu_baseline"].items() if k in SUB_CPU}
        out[name] = line
    if isinstance(cpu, dict) and "sample" in cpu:
        side["cpu_baseline"] = cpu
    if peak_of(tables):
        out["peak_clock_mhz"] = peak_of(tables).get("clock_mhz")
    if tables_out:
        try:
            os.makedirs(os.path.dirname(tables_out), exist_ok=True)
            with open(tables_out, "w") as f:
                json.dump(side, f, indent=1, default=str)
        except OSError as e:
            log("side file not written:", e)
    line = json.dumps(_round_floats(out))
    print(line, flush=True)
    return line


def _round_floats(x, sig=5):
    """floats to `sig` significant digits, recursively (the line's size, not its precision, is the limit)."""
    if isinstance(x, float):
        return float("%.*g" % (sig, x))
    if isinstance(x, dict):
        return {k: _round_floats(v, sig) for k, v in x.items()}
    if isinstance(x, list):
        return [_round_floats(v, sig) for v in x]
    return x


def peak_of(tables):
    return tables.get("peak") if isinstance(tables, dict) else None


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--global-rounds", type=int, default=0,
                    help="rounds per step over all GPUs (default 100k at N = 1, the 1M chain at N > 1)")
    ap.add_argument("--batch", type=int, default=0,
                    help="max rounds per device batch (default: the rank's whole range in one batch up to %d rounds, "
                         "so every rank runs the N = 1 step)" % MAX_BATCH)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--allow-unlinked", action="store_true",
                    help="without a digest-pinned chain file, measure GPU-signed unlinked rounds (labelled so in "
                         "`data`) instead of exiting with status 3")
    ap.add_argument("--sync", dest="use_sync", action="store_true",
                    help="blocking dg_verify_beacons_dev per batch (default: dg_verify_beacons_dev_async, so the "
                         "latency-bound tail of one batch overlaps the head of the next)")
    ap.add_argument("--tables-out", default=os.path.join(ROOT, "gpurun_out", "bench_tables.json"),
                    help="side file for the per-kernel timing tables and the peak probe details (rank 0)")
    ap.add_argument("--no-peak-detail", action="store_true",
                    help="measure only the roofline denominator, not the other probe forms (profiling runs)")
    ap.add_argument("--no-kernel-timing", action="store_true",
                    help="no per-kernel HIP events after the timed region (no roofline)")
    ap.add_argument("--recover-rounds", type=int, default=100000, help="C3 rounds (all GPUs); 0 disables")
    ap.add_argument("--c5-rounds", type=int, default=10000, help="C5 rounds (all GPUs); 0 disables")
    ap.add_argument("--sync-rounds", type=int, default=100000, help="0 disables the syncFrom catch-up line")
    ap.add_argument("--no-c1", action="store_true", help="no C1 / live-latency lines")
    ap.add_argument("--neg-steps", type=int, default=40,
                    help="steps of the c2_negative line (1%% of the signatures replaced); 0 disables.  A failed batch "
                         "lives ~90 ms on its tail queue, so 10 steps mostly time the pipeline filling and draining "
                         "(3.4 M rounds/s vs 3.8 M at 40, DESIGN.md §5.4)")
    ap.add_argument("--no-vp-negative", action="store_true", help="no vp_negative line (VerifyPartial on C5's set)")
    ap.add_argument("--status-bufs", type=int, default=int(os.environ.get("DG_SETS", "10")),
                    help="steps whose verdicts may be in flight (at least the library's workspace sets, DG_SETS = 10)")
    ap.add_argument("--hw-queues", type=int, default=int(os.environ.get("BENCH_HW_QUEUES", "0")),
                    help="HIP hardware queues per process (GPU_MAX_HW_QUEUES, set before HIP starts).  0 (default): "
                         "the environment's value, else the library's own load-time default (16: the library's 10 "
                         "workspace streams, its per-item stream and the caller's streams each want their own queue, "
                         "DESIGN.md §5.3)")
    args = ap.parse_args()
    if args.hw_queues > 0:
        os.environ["GPU_MAX_HW_QUEUES"] = str(args.hw_queues)  # inherited by the ranks started below

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # start the N ranks (one process per GPU) before anything in this process touches the GPU
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(args.gpus),
               "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.abspath(__file__)]
        cmd += sys.argv[1:]
        log("launching", " ".join(cmd))
        sys.exit(subprocess.call(cmd))
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log("world size %d != --gpus %d" % (world, args.gpus))
        sys.exit(2)
    # the chain before anything touches the GPU: no pinned file covering G rounds -> exit 3 (require_chain)
    G = args.global_rounds or (100000 if world == 1 else 1000000)
    chain = require_chain(G, args.allow_unlinked)
    # the library's load-time default of the hardware queue count (drand_gpu.hip dg_default_hw_queues: 16 unless the
    # process set GPU_MAX_HW_QUEUES) reaches a program linked against it before its first HIP call; here torch, which
    # brings its own HIP runtime, starts HIP and must start it first, so the bench applies the same default itself
    if args.hw_queues <= 0:
        os.environ.setdefault("GPU_MAX_HW_QUEUES", "16")
    hw_queues = int(os.environ["GPU_MAX_HW_QUEUES"])

    import torch
    import torch.distributed as dist

    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)

    from drand_amd import _lib as L
    from drand_amd import tbls, shard

    lib = L.lib(local)
    x = S.master_secret()
    pk = S.GROUP_PK  # x * g1, the chain's group key (public fixture constant)
    a, b = shard.round_range(G, world, rank)
    n = b - a
    if chain is not None:
        sigs = chain[a:b]
        prev = chain[a - 1:b - 1] if a > 0 else np.concatenate([np.zeros((1, 96), np.uint8), chain[:b - 1]])
        data = "synthetic linked chain data/chain_v1 (CPU-twin generated, seed tools/synthetic.py)"
        linked = True
    else:
        prev, sigs = gpu_signed_rounds(tbls, a + 1, n, x)
        data = "synthetic rounds, GPU-signed (no chain file: prev_sig pseudo-random, links not checked)"
        linked = False
    bounds = batch_bounds(n, args.batch)
    nb = len(bounds)
    mbytes = (max(y - x_ for x_, y in (shard.round_range(G, world, q) for q in range(world))) + 7) // 8
    rounds = np.arange(a + 1, b + 1, dtype=np.uint64)
    prev_sigs = [bytes(p) for p in prev]
    if a == 0 and linked:
        prev_sigs[0] = S.GENESIS_SEED
    _, _, psb, off = tbls._beacon_arrays(rounds - 1, rounds, prev_sigs)
    d_pr = torch.from_numpy((rounds - 1).astype(np.int64)).to(dev)
    d_r = torch.from_numpy(rounds.astype(np.int64)).to(dev)
    d_ps = torch.from_numpy(psb).to(dev)
    d_off = torch.from_numpy(off.astype(np.int32)).to(dev)
    d_sig = torch.from_numpy(np.ascontiguousarray(sigs)).to(dev)
    # status buffers rotate over the steps in flight (the library itself keeps at most DG_SETS = 10 batches
    # in flight); a buffer is reused once the all-gather that read it has finished
    nbuf = args.status_bufs
    d_sts = [torch.full((n,), 99, dtype=torch.uint8, device=dev) for _ in range(nbuf)]
    gathered = [None] * nbuf
    side = torch.cuda.Stream(dev)
    pkb = ctypes.c_char_p(pk)
    counter = [0]

    # one batch per step on one rank: the verdict bitmap is packed on the batch's own stream (dg_last_batch_stream), so
    # no cross-stream wait is queued -- with HIP's default 4 hardware queues a wait on a queue shared with another
    # workspace set stalls that set; several batches or ranks: a side stream waits for them all
    on_set = consume_on_batch_stream(len(bounds), args.use_sync)

    sig_src = [d_sig]  # the signatures the steps verify (the c2_negative line swaps in a corrupted copy)

    hostprof = collections.defaultdict(float) if os.environ.get("DG_BENCH_HOSTPROF") else None
    # BENCH_STEP_TIMES=1 (diagnostics): each timed step's completion (its bitmap's event) in ms from the region's start,
    # on stderr -- the pipeline's fill, steady spacing and drain
    step_times = None

    def enqueue(lo, hi, d_st, seed, blocking):
        args_ = (pkb, hi - lo, L.ptr(d_pr[lo:]), L.ptr(d_r[lo:]), L.ptr(d_ps), L.ptr(d_off[lo:]),
                 L.ptr(sig_src[0][lo:]), L.ptr(d_st[lo:]), seed)
        h0 = time.perf_counter()
        if blocking:
            L.check(lib.dg_verify_beacons_dev(*args_, None))
        else:
            L.check(lib.dg_verify_beacons_dev_async(*args_, None, None if on_set else ctypes.c_void_p(side.cuda_stream)))
        if hostprof is not None:
            hostprof["enqueue_s"] += time.perf_counter() - h0
            hostprof["enqueues"] += 1

    def step(seed):
        """Enqueue this rank's batches (asynchronously: consecutive batches overlap) and the all-gather of the
        rank's verdict bitmap on a stream that follows them; returns the gathered bitmap tensor."""
        i = counter[0] % nbuf
        counter[0] += 1
        if gathered[i] is not None:
            h0 = time.perf_counter()
            gathered[i][1].synchronize()  # the all-gather that read this status buffer has finished
            if hostprof is not None:
                hostprof["bufwait_s"] += time.perf_counter() - h0
        d_st = d_sts[i]
        for j, (lo, hi) in enumerate(bounds):
            enqueue(lo, hi, d_st, seed * 64 + j, args.use_sync)
        if args.use_sync:
            side.wait_stream(torch.cuda.current_stream(dev))
        gs = side
        if on_set:
            sp = ctypes.c_void_p()
            L.check(lib.dg_last_batch_stream(ctypes.byref(sp)))
            gs = torch.cuda.ExternalStream(sp.value, device=dev)
        with torch.cuda.stream(gs):
            bits = shard.allgather_verdicts(d_st, world, m=mbytes)
            ev = torch.cuda.Event(enable_timing=step_times is not None)
            ev.record(gs)
        gathered[i] = (bits, ev)
        if step_times is not None:
            step_times.append(ev)
        return bits

    def drain():
        L.check(lib.dg_wait_all())
        torch.cuda.synchronize()

    # prime every workspace set once (its grow-only buffers are allocated on first use), then the W warmup
    # steps: no allocation or first-dispatch cost falls inside the timed region
    for w in range(max(1, int(os.environ.get("DG_SETS", "10")) // nb + 1)):
        step(500 + w)
    drain()
    for w in range(args.warmup):
        step(1000 + w)
    drain()
    bitmap = step(7)
    drain()
    assert all(int(d.max().item()) == 0 for d in d_sts[:min(counter[0], nbuf)]), "valid chain rounds rejected"
    assert bitmap.sum().item() == 0
    if world > 1:
        dist.barrier()
    L.check(lib.dg_set_timing(0))  # no per-kernel events inside the timed region
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    fb0 = L.fallback_count()
    ev0 = None
    if os.environ.get("BENCH_STEP_TIMES"):
        step_times = []
        ev0 = torch.cuda.Event(enable_timing=True)
        ev0.record(torch.cuda.current_stream(dev))
    t0 = time.perf_counter()
    if hostprof is not None:
        hostprof.clear()
    bits = [step(17 + s) for s in range(args.steps)]
    if hostprof is not None:
        hostprof["steps_enqueued_s"] = time.perf_counter() - t0
    drain()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    if ev0 is not None:
        ts = [round(ev0.elapsed_time(e), 3) for e in step_times]
        print("[step_times] region %.3f ms, completions (ms): %s" % (dt * 1e3, ts), file=sys.stderr, flush=True)
        step_times = None
    if hostprof is not None:
        hostprof["timed_s"] = dt
        print("[hostprof]", json.dumps({k: round(v, 5) for k, v in hostprof.items()}), file=sys.stderr, flush=True)
    assert all(int(bt.sum().item()) == 0 for bt in bits)
    assert all(int(d.max().item()) == 0 for d in d_sts[:min(counter[0], nbuf)])  # (buffers no step used hold 99)
    fallbacks = L.fallback_count() - fb0  # timed batches that ran the per-item pass (0 for valid chains)
    # instrumented replay of the timed region (same steps, same seeds) with HIP events around every launch on
    # its stream: per-kernel averages while the batches overlap; then one batch through the blocking entry
    # point, so each kernel runs alone on the chip
    kt, kt_iso = {}, {}
    if not args.no_kernel_timing:
        L.check(lib.dg_set_timing(1))
        [step(17 + s) for s in range(args.steps)]
        drain()
        kt = L.timings()
        L.check(lib.dg_set_timing(0))
        L.check(lib.dg_set_timing(1))
        lo, hi = bounds[0]
        for s in range(2):
            enqueue(lo, hi, d_sts[0], 900 + s, True)
        kt_iso = L.timings()
        assert int(d_sts[0][lo:hi].max().item()) == 0
        L.check(lib.dg_set_timing(0))
    dt = max_over_ranks(dt, world)
    # every rank measures the v_mad_u64_u32 peak of its own GPU: the Recover lines below price their kernels
    # against it on every rank
    peak = measure_peak(shard, local, detail=(rank == 0 and not args.no_peak_detail))
    roof = headline_roofline(kt, kt_iso, bounds[0][1] - bounds[0][0], peak, G, args.steps, world, dt)
    share = {k: round(v[0] * v[1] / (dt * 1e6), 4) for k, v in kt.items()}
    neg = None
    if args.neg_steps > 0:
        neg = negative_bench(L, args, step, drain, sig_src, d_sts, nbuf, counter, n, a, G, world, peak, bounds)
    del d_sts, d_sig, d_ps
    torch.cuda.empty_cache()

    # Recover lines (sharded like the headline; chain rounds 1..R)
    rec = adv = syn = c1 = lat = c2 = vpn = None
    rec_in = adv_in = None
    src = None
    if args.recover_rounds or args.c5_rounds or args.sync_rounds:
        src = RoundSource(tbls, max(args.recover_rounds, args.c5_rounds + 1, args.sync_rounds, 1000),
                          args.allow_unlinked)
    if args.recover_rounds:
        rec, rec_in, c2 = recover_bench(L, tbls, shard, src, args.recover_rounds, 33, 64, world, rank, peak)
    if args.c5_rounds:
        adv, adv_in, vpn = adversarial_bench(L, tbls, shard, src, args.c5_rounds, world, rank, peak,
                                             vp_neg=not args.no_vp_negative)
    if rank == 0:
        if args.sync_rounds and src.linked:
            syn = sync_bench(src.sigs, args.sync_rounds)
        if not args.no_c1:
            c1 = c1_gpu(L, tbls)
            if rec_in is not None:
                lat = live_latency(L, tbls, rec_in[0], rec_in[1], rec_in[2], 33, 64)
    # CPU baselines: rank 0 at every N, after every GPU timed region, on all the host cores it may use
    cpu = None
    if rank == 0 and not args.no_cpu_baseline:
        th, machine, quota = host_cores()
        ns = min(n, 40000)
        m = tbls.beacon_messages(rounds[:ns] - 1, rounds[:ns], prev_sigs[:ns])
        cpu = cpu_label(cpu_verify(pk, m, np.ascontiguousarray(sigs[:ns]), th), th, machine, quota)
        if c1 is not None:
            c1["cpu_baseline"] = cpu_label(cpu_c1(th), th, machine, quota)
        if rec_in is not None:
            cb, _ = cpu_recover(rec_in[0], 33, 64, rec_in[1], rec_in[2], th, label="C3 n=64 t=33")
            rec["cpu_baseline"] = cpu_label(cb, th, machine, quota)
            if c2 is not None:
                # configs[2] on the host: every partial VerifyPartial'd, then kyber's Recover
                vps, vsample = cpu_verify_partials(rec_in[0], rec_in[1], rec_in[2], th)
                c2["cpu_baseline"] = cpu_label({"value": 1.0 / (64 / vps + 1.0 / cb["value"]), "unit": "recovers/s",
                                                "kind": "port", "partials_verified_per_s": vps,
                                                "sample": vsample + "; Recover: " + cb["sample"]}, th, machine, quota)
        if adv_in is not None:
            cb, (trs, tss, Rs) = cpu_recover(adv_in[0], 129, 256, adv_in[1], adv_in[2], th, seconds=6.0,
                                             label="C5 n=256 t=129 corrupted")
            # the GPU's statuses on the same rounds are the twin's (bit-exact sample check)
            cb["statuses_match_gpu"] = bool(np.array_equal(tss, adv_in[3][:Rs]) and np.array_equal(trs, adv_in[4][:Rs]))
            adv["cpu_baseline"] = cpu_label(cb, th, machine, quota)
    head = {"value": G * args.steps / dt, "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": dt / args.steps * 1e3,
            "scaling": "strong" if (world > 1 or args.global_rounds) else "weak", "data": data,
            "config": {"workload": ("batch bls.Verify / beacon.VerifyBeacon of the %d-round linked chain per "
                                    "step, %d contiguous range(s) of <= %d rounds per GPU in batches of <= %d, "
                                    "one shared group key (BASELINE configs[%d])"
                                    % (G, world, -(-G // world), max(y - x_ for x_, y in bounds),
                                       1 if G <= 100000 else 3)),
                       "global_rounds": G, "rounds_per_gpu": n, "batches_per_gpu": nb,
                       "hip_hw_queues": hw_queues,
                       "parallelism": "rounds sharded dp%d" % world},
            "batch_fallbacks": fallbacks}
    tables = {"kernel_time_share": share, "kernel_avg_us": {k: round(v[0], 1) for k, v in kt.items()},
              "kernel_avg_us_isolated": {k: round(v[0], 1) for k, v in kt_iso.items()}, "peak": peak}
    report(rank, world, head, roof, cpu, {"recover": rec, "adversarial": adv, "c1": c1, "live_latency": lat,
                                          "sync": syn, "c2_verify_all": c2, "c2_negative": neg,
                                          "vp_negative": vpn}, tables, args.tables_out)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
