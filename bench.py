"""Benchmark of the threshold-BLS hot path (BASELINE.json): verified beacon rounds/s.

A step = one dg_verify_beacons_dev pass over this rank's contiguous range of the synthetic linked chain
(beacon.Message on the device, hash-to-G2, sigma decode + subgroup check, RLC multi-pairing with one
shared final exponentiation; BASELINE configs[1] at N = 1: 100k rounds, one shared group key), inputs
resident in HBM, followed by the RCCL all-gather of the per-round verdict bitmaps (configs[3] at N > 1,
one contiguous round range per GPU, weak scaling).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--rounds R] [--no-cpu-baseline]

Rank 0 prints ONE JSON line (contract in the task statement); the roofline object is the integer
multiply-add rate of the dominant kernel (algorithmic MACs from profiles/opcounts.json / its average
HIP-event duration measured live on the launch stream) against the measured v_mad_u64_u32 peak.
"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from tools import synthetic as S  # noqa: E402

METRIC = "verified beacon rounds/sec (pairing checks/s)"


def log(*a):
    print("[bench]", *a, file=sys.stderr, flush=True)


def traffic_of(kernel):
    """HBM-side bytes per launch of `kernel` from the committed PMC passes (profiles/traffic.json, made by
    tools/traffic.py from separate rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE runs of this bench): 2 x
    FETCH_SIZE + WRITE_SIZE (the gfx950 correction of FETCH_SIZE), or None without a profile."""
    p = os.path.join(ROOT, "profiles", "traffic.json")
    if not os.path.exists(p):
        return None
    t = json.load(open(p)).get("kernels", {}).get(kernel)
    return t["bytes_per_launch"] if t else None


def load_chain(total):
    """(sigs (total, 96), prev_sig of round 1) for rounds 1..total of the synthetic chain."""
    best = None
    d = os.path.join(ROOT, "data")
    if os.path.isdir(d):
        for f in os.listdir(d):
            if f.startswith("chain_v1_") and f.endswith(".bin"):
                n = int(f[len("chain_v1_"):-4])
                if n >= total and (best is None or n < best[0]):
                    best = (n, os.path.join(d, f))
    if best is None:
        return None
    mm = np.memmap(best[1], dtype=np.uint8, mode="r", shape=(best[0], 96))
    return np.array(mm[:total])


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


def cpu_baseline(pk, msgs, sigs, seconds=10.0, threads=16):
    """The CPU twin (C port of the reference algorithm: one full pairing check per beacon) on a bounded
    sample of the same rounds, `threads` POSIX threads."""
    from oracle import twin

    n0 = 64
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


def recover_bench(L, tbls, chain_sigs, first_round, R, t, n, steps):
    """BASELINE configs[2]: VerifyPartial on every share + Lagrange Recover for an (n, t) group
    over R rounds of the chain, through dg_recover (host-buffer API: the 98 B partials cross PCIe inside the
    timed region).  Partials are produced on the GPU by dg_sign (untimed); every recovered signature must
    equal the chain's signature byte for byte."""
    g = json.load(open(os.path.join(ROOT, "tests", "golden", "groups.json")))["t%d" % t]
    pub = tbls.PubPoly([bytes.fromhex(c) for c in g])
    coeffs = S.poly_coeffs(t)
    shares = [S.share_value(coeffs, i) for i in range(n)]
    rounds = np.arange(first_round, first_round + R, dtype=np.uint64)
    prev = [bytes(chain_sigs[r - 2]) if r >= 2 else S.GENESIS_SEED for r in rounds.tolist()]
    msgs = tbls.beacon_messages(rounds - 1, rounds, prev)
    sc = [shares[i] for _ in range(R) for i in range(n)]
    idx = [i for _ in range(R) for i in range(n)]
    t0 = time.perf_counter()
    parts = tbls.sign_batch(sc, np.repeat(msgs, n, axis=0), idx).reshape(R, n, 98)
    gen_s = time.perf_counter() - t0
    sigs, rs, ss = tbls.recover_batch(pub, msgs, parts, t, n, seed=5)  # warmup + check
    want = chain_sigs[first_round - 1:first_round - 1 + R]
    assert not rs.any() and np.array_equal(sigs, want), "recovered signatures differ from the chain"
    t0 = time.perf_counter()
    for s in range(steps):
        tbls.recover_batch(pub, msgs, parts, t, n, seed=6 + s)
    dt = (time.perf_counter() - t0) / steps
    return {"metric": "Recover/s at n=%d t=%d (all %d shares VerifyPartial'd, first t valid interpolated)" % (n, t, n),
            "value": R / dt, "unit": "recovers/s", "rounds": R, "partials_per_round": n, "s_per_step": dt,
            "partials_verified_per_s": R * n / dt, "partials_generated_s": gen_s,
            "note": "host-buffer C-ABI (dg_recover): PCIe transfer of %d MB of partials inside the timed region; "
                    "recovered signatures equal the chain's" % (R * n * 98 // 10**6)}


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


def adversarial_bench(L, tbls, chain_sigs, R, t=129, n=256, frac=0.10, n_short=3):
    """BASELINE configs C5: n = 256, t = 129, R rounds, ~10% of the (round, share) cells
    corrupted with the six cycling modes of tools/corrupt.py, plus `n_short` rounds with more than n - t
    corrupted shares (-> "not enough shares").  One dg_recover over all R x n partials (VerifyPartial on
    every share -- the batch equation fails, so every share takes the exact per-item check -- then
    Recover).  Checked without the CPU: recovered signatures equal the chain's, exactly the short rounds
    report NOT_ENOUGH, every examined corrupted share is rejected and every examined clean one accepted
    (per-share parity with the CPU twin is tests/test_gpu_parity.py's job)."""
    from tools import corrupt

    g = json.load(open(os.path.join(ROOT, "tests", "golden", "groups.json")))["t%d" % t]
    pub = tbls.PubPoly([bytes.fromhex(c) for c in g])
    coeffs = S.poly_coeffs(t)
    shares = [S.share_value(coeffs, i) for i in range(n)]
    rounds = np.arange(1, R + 2, dtype=np.uint64)  # one extra round for the "other_round" mode
    prev = [S.GENESIS_SEED] + [bytes(chain_sigs[r - 2]) for r in rounds.tolist()[1:]]
    msgs_all = tbls.beacon_messages(rounds - 1, rounds, prev)
    msgs = msgs_all[:R]
    t0 = time.perf_counter()
    parts = tbls.sign_batch([shares[i] for _ in range(R) for i in range(n)], np.repeat(msgs, n, axis=0),
                            [i for _ in range(R) for i in range(n)]).reshape(R, n, 98)
    items = corrupt.pick(R, n, frac)
    short = set(range(n_short))
    items = [it for it in items if it[0] not in short] + [(r, j, "random_bytes") for r in short
                                                           for j in range(n - t + 2)]

    def resign(reqs):
        sc = [shares[idx] + ds for _, idx, ds, _ in reqs]
        return tbls.sign_batch(sc, np.stack([msgs_all[r + dr] for r, _, _, dr in reqs]))

    corrupt.corrupt_batch(parts, items, n, resign)
    gen_s = time.perf_counter() - t0
    bad = np.zeros((R, n), dtype=bool)
    for r, j, _ in items:
        bad[r, j] = True
    sigs, rs, ss = tbls.recover_batch(pub, msgs, parts, t, n, seed=11)  # warmup + check
    ok_r = np.array([r not in short for r in range(R)])
    assert np.array_equal(rs != 0, ~ok_r) and (rs[~ok_r] == 5).all(), "round statuses"
    assert np.array_equal(sigs[ok_r], chain_sigs[:R][ok_r]), "recovered signatures differ from the chain"
    examined = ss != 255
    assert (ss[examined & bad] != 0).all() and (ss[examined & ~bad] == 0).all(), "share statuses"
    t0 = time.perf_counter()
    tbls.recover_batch(pub, msgs, parts, t, n, seed=12)
    dt = time.perf_counter() - t0
    return {"metric": "adversarial Recover/s at n=%d t=%d, %.0f%% of shares corrupted (C5)" % (n, t, 100 * frac),
            "value": R / dt, "unit": "recovers/s", "rounds": R, "partials_per_round": n,
            "corrupted_shares": int(bad.sum()), "short_rounds": n_short, "s_per_step": dt,
            "partials_verified_per_s": R * n / dt, "setup_s": gen_s,
            "note": "host-buffer C-ABI (dg_recover), PCIe transfer of %d MB of partials inside the timed region; "
                    "every batch fails its RLC check, so all shares take the per-item pairing check"
                    % (R * n * 98 // 10**6)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--rounds", type=int, default=100000, help="rounds per GPU per step")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-threads", type=int, default=16)
    ap.add_argument("--sync", dest="use_sync", action="store_true",
                    help="blocking dg_verify_beacons_dev per step (default: dg_verify_beacons_dev_async, so the "
                         "latency-bound tail of one batch overlaps the head of the next)")
    ap.add_argument("--no-kernel-timing", action="store_true",
                    help="no per-kernel HIP events in the timed region (no roofline)")
    ap.add_argument("--recover-rounds", type=int, default=20000, help="0 disables the Recover line")
    ap.add_argument("--c5-rounds", type=int, default=10000, help="0 disables the adversarial (C5) line")
    ap.add_argument("--sync-rounds", type=int, default=100000, help="0 disables the syncFrom catch-up line")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)

    from drand_amd import _lib as L
    from drand_amd import tbls, shard

    lib = L.lib(local)
    R = args.rounds
    x = S.master_secret()
    pk = S.GROUP_PK  # x * g1, the chain's group key (public fixture constant)
    a, b = shard.round_range(world * R, world, rank)
    chain = load_chain(world * R)
    if chain is not None:
        sigs = chain[a:b]
        prev = chain[a - 1:b - 1] if a > 0 else np.concatenate([np.zeros((1, 96), np.uint8), chain[:b - 1]])
        data = "synthetic linked chain data/chain_v1 (CPU-twin generated, seed tools/synthetic.py)"
        linked = True
    else:
        prev, sigs = gpu_signed_rounds(tbls, a + 1, b - a, x)
        data = "synthetic rounds, GPU-signed (no chain file: prev_sig pseudo-random, links not checked)"
        linked = False
    n = b - a
    mbytes = (max(y - x for x, y in (shard.round_range(world * R, world, q) for q in range(world))) + 7) // 8
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
    # one status buffer per in-flight batch (the library rotates over DG_SETS = 4 workspace sets)
    nbuf = 4
    d_sts = [torch.full((n,), 99, dtype=torch.uint8, device=dev) for _ in range(nbuf)]
    gathered = [None] * nbuf
    side = torch.cuda.Stream(dev)
    pkb = ctypes.c_char_p(pk)
    counter = [0]

    def step(seed):
        """Enqueue one batch (asynchronously: consecutive batches overlap) and the all-gather of its verdict
        bitmap on a side stream that waits for the batch; returns the gathered bitmap tensor."""
        i = counter[0] % nbuf
        counter[0] += 1
        if gathered[i] is not None:
            gathered[i][1].synchronize()  # the all-gather that read this status buffer has finished
        d_st = d_sts[i]
        if args.use_sync:
            L.check(lib.dg_verify_beacons_dev(pkb, n, L.ptr(d_pr), L.ptr(d_r), L.ptr(d_ps), L.ptr(d_off),
                                              L.ptr(d_sig), L.ptr(d_st), seed, None))
            side.wait_stream(torch.cuda.current_stream(dev))
        else:
            L.check(lib.dg_verify_beacons_dev_async(pkb, n, L.ptr(d_pr), L.ptr(d_r), L.ptr(d_ps), L.ptr(d_off),
                                                    L.ptr(d_sig), L.ptr(d_st), seed, None,
                                                    ctypes.c_void_p(side.cuda_stream)))
        with torch.cuda.stream(side):
            bits = shard.allgather_verdicts(d_st, world, m=mbytes)
            ev = torch.cuda.Event()
            ev.record(side)
        gathered[i] = (bits, ev)
        return bits

    def drain():
        L.check(lib.dg_wait_all())
        torch.cuda.synchronize()

    # prime every workspace set once (its grow-only buffers are allocated on first use), then the W warmup
    # steps: no allocation or first-dispatch cost falls inside the timed region
    for w in range(nbuf):
        step(500 + w)
    drain()
    for w in range(args.warmup):
        step(1000 + w)
    drain()
    bitmap = step(7)
    drain()
    used = min(counter[0], nbuf)
    assert all(int(d.max().item()) == 0 for d in d_sts[:used]), "valid chain rounds rejected"
    assert bitmap.sum().item() == 0
    if world > 1:
        dist.barrier()
    L.check(lib.dg_set_timing(0))  # no per-kernel events inside the timed region
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    fb0 = L.fallback_count()
    t0 = time.perf_counter()
    bits = [step(17 + s) for s in range(args.steps)]
    drain()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    used = min(counter[0], nbuf)
    assert all(int(b.sum().item()) == 0 for b in bits) and all(int(d.max().item()) == 0 for d in d_sts[:used])
    fallbacks = L.fallback_count() - fb0  # timed batches that ran the per-item pass (0 for valid chains)
    # instrumented replay of the timed region (same steps, same seeds) with HIP events around every
    # launch on its stream: per-kernel averages while the batches overlap
    kt, kt_iso = {}, {}
    if not args.no_kernel_timing:
        L.check(lib.dg_set_timing(1))
        [step(17 + s) for s in range(args.steps)]
        drain()
        kt = L.timings()
        # the same batch through the blocking entry point, so each kernel runs alone on the chip
        L.check(lib.dg_set_timing(0))
        L.check(lib.dg_set_timing(1))
        for s in range(2):
            L.check(lib.dg_verify_beacons_dev(pkb, n, L.ptr(d_pr), L.ptr(d_r), L.ptr(d_ps), L.ptr(d_off),
                                              L.ptr(d_sig), L.ptr(d_sts[0]), 900 + s, None))
        kt_iso = L.timings()
        assert int(d_sts[0].max().item()) == 0
        L.check(lib.dg_set_timing(0))
    t = torch.tensor([dt], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    dt = float(t.item())
    total = world * n * args.steps
    if rank == 0:
        oc = json.load(open(os.path.join(ROOT, "profiles", "opcounts.json")))["per_unit"]
        # dominant kernel by its isolated time (blocking batches after the timed region, one kernel on the
        # chip at a time -- the launches rocprofv3 --stats of `bench.py --sync` averages); the same kernel's
        # average inside the overlapped timed region is reported beside it
        src = kt_iso if kt_iso else kt
        name, (us, launches) = max(src.items(), key=lambda kv: kv[1][0] * kv[1][1]) if src else (None, (0, 0))
        per_launch_units = n
        macs = oc.get(name, {}).get("macs") if name else None
        peak = shard.mad_peak()
        roof = None
        if macs is not None:
            achieved = macs * per_launch_units / (us * 1e-6) / 1e12
            roof = {"bound": "valu-int", "achieved": achieved, "peak": peak["tmac_s"], "unit": "TMAC/s",
                    "frac": achieved / peak["tmac_s"], "traffic": traffic_of(name), "kernel": name,
                    "kernel_avg_us": us, "units_per_launch": per_launch_units, "macs_per_unit": macs,
                    "peak_source": peak["source"],
                    "timing": "HIP events on the launch stream, blocking batches right after the timed region "
                              "(the kernel alone on the chip)"}
            if name in kt:
                o_us = kt[name][0]
                a_o = macs * per_launch_units / (o_us * 1e-6) / 1e12
                roof["overlapped"] = {"kernel_avg_us": o_us, "achieved": a_o, "frac": a_o / peak["tmac_s"],
                                      "note": "instrumented replay of the timed region: the launch shares the "
                                              "chip with the other batches in flight"}
            # whole chip: algorithmic multiply-adds of the per-round work (hash, decode, 16 bucket additions
            # of the two MSMs + 10 of the subgroup-check test windows, mixed: signatures and hashes are
            # stored with Z = 1) over the step time; per-batch fixed work not counted
            per_round = (sum(oc[k]["macs"] for k in ("k_h2c_uncleared", "k_decode_items")) +
                         26 * oc["k_msm_chunks[mixed add]"]["macs"])
            chip = per_round * n * args.steps / dt / 1e12
            roof["chip"] = {"macs_per_round": per_round, "achieved": chip, "frac": chip / peak["tmac_s"]}
        share = {k: round(v[0] * v[1] / (dt * 1e6 / 1.0), 4) for k, v in kt.items()}
        rec = None
        if args.recover_rounds and chain is not None:
            rec = recover_bench(L, tbls, chain, 1, min(args.recover_rounds, len(chain)), 33, 64, 1)
        adv = None
        if args.c5_rounds and chain is not None:
            adv = adversarial_bench(L, tbls, chain, min(args.c5_rounds, len(chain) - 1))
        syn = None
        if args.sync_rounds and chain is not None:
            syn = sync_bench(chain, min(args.sync_rounds, len(chain)))
        cpu = None
        if not args.no_cpu_baseline:
            ns = min(n, 40000)  # the sampler stops at ~10 s of 16-thread CPU work
            m = tbls.beacon_messages(rounds[:ns] - 1, rounds[:ns], prev_sigs[:ns])
            cpu = cpu_baseline(pk, m, np.ascontiguousarray(sigs[:ns]), threads=args.cpu_threads)
        out = {"metric": METRIC, "value": total / dt, "unit": "rounds/s", "n_gpus": world, "steps": args.steps,
               "warmup": args.warmup, "ms_per_step": dt / args.steps * 1e3, "higher_is_better": True,
               "scaling": "weak", "vs_baseline": None, "dtype": "u32 (381-bit Fp, 12x32-bit limbs)", "data": data,
               "config": {"workload": "batch bls.Verify / beacon.VerifyBeacon of %d linked chain rounds per GPU, one "
                                      "shared group key (BASELINE configs[1]; configs[3] at N>1)" % n,
                          "rounds_per_gpu": n, "global_rounds": world * n, "parallelism": "rounds sharded dp%d" % world},
               "roofline": roof, "cpu_baseline": cpu, "recover": rec, "adversarial": adv, "sync": syn,
               "batch_fallbacks": fallbacks,
               "kernel_time_share": share,
               "kernel_avg_us": {k: round(v[0], 1) for k, v in kt.items()},
               "kernel_avg_us_isolated": {k: round(v[0], 1) for k, v in kt_iso.items()}}
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
