"""Multi-GPU layout of the verify path: one process per GPU, one contiguous round range
per rank, no data-path collective; the only exchange is the all-gather of the per-round results --
verdict bitmaps (VerifyBeacon), recovered signatures, round statuses and per-share statuses (Recover)
-- over RCCL/xGMI on the GPU node, gloo in the CPU tests."""
import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
PROBE = os.path.join(os.path.dirname(_HERE), "tools", "microbench", "libdrandprobe.so")


def round_range(total, world, rank):
    """[a, b) of `total` rounds for `rank`: contiguous, sizes differ by at most one."""
    base, extra = divmod(total, world)
    a = rank * base + min(rank, extra)
    return a, a + base + (1 if rank < extra else 0)


def pack_bits(status):
    """uint8 status per round (torch tensor) -> verdict bitmap (1 = rejected), little-endian bit order."""
    import torch

    bad = (status != 0).to(torch.uint8)
    pad = (-bad.numel()) % 8
    if pad:
        bad = torch.cat([bad, torch.zeros(pad, dtype=torch.uint8, device=bad.device)])
    # bit weights made on the device (a host-built tensor would be a blocking copy on the current stream,
    # which serialises it with the batch it waits for)
    shift = torch.arange(8, dtype=torch.uint8, device=bad.device)
    return (bad.view(-1, 8) << shift).sum(dim=1).to(torch.uint8)


def allgather_verdicts(status, world, group=None, m=None):
    """All-gather every rank's packed verdict bitmap (equal-size shards padded to the largest).

    m = bitmap bytes of the largest shard; when the caller knows it (round_range makes the shard sizes a
    function of the global size), no host round trip is needed and the gather stays stream-ordered."""
    import torch
    import torch.distributed as dist

    bits = pack_bits(status)
    if world == 1:
        return bits
    if m is None:
        n = torch.tensor([bits.numel()], device=bits.device, dtype=torch.int64)
        dist.all_reduce(n, op=dist.ReduceOp.MAX, group=group)
        m = int(n.item())
    if bits.numel() < m:
        bits = torch.cat([bits, torch.zeros(m - bits.numel(), dtype=torch.uint8, device=bits.device)])
    if dist.get_backend(group) == "nccl":  # RCCL on ROCm
        out = torch.empty(world * m, dtype=torch.uint8, device=bits.device)
        dist.all_gather_into_tensor(out, bits, group=group)
        return out
    parts = [torch.empty(m, dtype=torch.uint8, device=bits.device) for _ in range(world)]
    dist.all_gather(parts, bits, group=group)  # gloo (CPU tests)
    return torch.cat(parts)


def allgather_rows(rows, world, total, group=None):
    """All-gather a rank's contiguous block of per-round records (a (n_rank, w) uint8 tensor, rank r holding
    rounds round_range(total, world, r)) into the (total, w) array of every round, in round order.

    Shards are padded to the largest one (its size is a function of `total`, so no size exchange and no host
    round trip); one all_gather_into_tensor on RCCL, list all_gather on gloo.  Used for the Recover outputs:
    96 B recovered signatures, the round status byte and the k share-status bytes of every round."""
    import torch
    import torch.distributed as dist

    if rows.dim() == 1:
        rows = rows.view(-1, 1)
    w = rows.shape[1]
    sizes = [b - a for a, b in (round_range(total, world, q) for q in range(world))]
    if world == 1:
        return rows
    m = max(sizes)
    if rows.shape[0] < m:
        rows = torch.cat([rows, torch.zeros((m - rows.shape[0], w), dtype=rows.dtype, device=rows.device)])
    rows = rows.contiguous()
    if dist.get_backend(group) == "nccl":  # RCCL on ROCm
        out = torch.empty((world * m, w), dtype=rows.dtype, device=rows.device)
        dist.all_gather_into_tensor(out, rows, group=group)
    else:
        parts = [torch.empty((m, w), dtype=rows.dtype, device=rows.device) for _ in range(world)]
        dist.all_gather(parts, rows, group=group)
        out = torch.cat(parts)
    return torch.cat([out[q * m:q * m + sizes[q]] for q in range(world)])


def unpack_bits(bitmap, sizes):
    """Inverse of the padded all-gather: per-rank bitmaps -> one flat verdict array (numpy)."""
    b = np.unpackbits(np.asarray(bitmap, dtype=np.uint8), bitorder="little")
    m = len(b) // len(sizes)
    return np.concatenate([b[r * m:r * m + s] for r, s in enumerate(sizes)])


def probe_form(device, kind, warm_s=2.0):
    """One form of the peak probe (tools/microbench/probe.hip kinds): lane-ops/s after warm_s seconds of
    launches, the in-kernel clock, and the SIMD cycles per wave64 instruction that implies."""
    lib = ctypes.CDLL(PROBE)
    rate = ctypes.c_double()
    mhz = ctypes.c_double()
    cus = ctypes.c_int()
    rc = lib.probe_run(device, kind, ctypes.c_double(warm_s), ctypes.byref(rate), ctypes.byref(mhz),
                       ctypes.byref(cus))
    if rc != 0:
        raise RuntimeError("probe_run failed")
    simd_cycles = cus.value * 4 * mhz.value * 1e6
    return {"tops": rate.value / 1e12, "clock_mhz": mhz.value, "cus": cus.value,
            "cycles_per_wave_instr": simd_cycles / (rate.value / 64.0) if rate.value else None}


def mad_peak(device=0):
    """Measured v_mad_u64_u32 lane-MAC rate (the integer-VALU roofline denominator): eight independent chains
    per lane with distinct carry destinations, timed after 2 s of back-to-back launches, with the clock the
    chip held; and the spec-rate ceiling at 2.4 GHz for the measured cycles per instruction."""
    f = probe_form(device, 1, warm_s=2.0)
    cyc = f["cycles_per_wave_instr"]
    spec = f["cus"] * 4 * 2.4e9 * 64 / round(cyc) / 1e12 if cyc else None
    return {"tmac_s": f["tops"], "cus": f["cus"], "clock_mhz": f["clock_mhz"], "cycles_per_wave_instr": cyc,
            "spec_tmac_s_at_2400mhz": spec,
            "source": "measured: 8 independent v_mad_u64_u32 chains per lane, distinct SGPR carry destinations, "
                      "after 2 s of launches (tools/microbench/probe.hip kind 1), %d CUs at %.0f MHz in-kernel"
                      % (f["cus"], f["clock_mhz"])}
