"""Multi-GPU layout on the CPU (gloo, world size 2): contiguous round ranges and the all-gather of
verdict bitmaps, the only exchange of the sharded verify path."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from drand_amd import shard


def test_round_range_partitions():
    for total in (0, 1, 7, 100000, 1000000):
        for world in (1, 2, 3, 4, 8):
            got = [shard.round_range(total, world, r) for r in range(world)]
            assert got[0][0] == 0 and got[-1][1] == total
            assert all(got[i][1] == got[i + 1][0] for i in range(world - 1))
            sizes = [b - a for a, b in got]
            assert max(sizes) - min(sizes) <= 1


def test_pack_unpack_bits():
    st = torch.tensor([0, 1, 0, 0, 2, 0, 0, 0, 0, 5, 0], dtype=torch.uint8)
    bits = shard.pack_bits(st)
    assert bits.numel() == 2
    flat = shard.unpack_bits(bits.numpy(), [11])
    assert flat.tolist() == [0, 1, 0, 0, 1, 0, 0, 0, 0, 1, 0]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, total, bad, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    a, b = shard.round_range(total, world, rank)
    st = torch.zeros(b - a, dtype=torch.uint8)
    for r in bad:
        if a <= r < b:
            st[r - a] = 1
    out = shard.allgather_verdicts(st, world)
    sizes = [y - x for x, y in (shard.round_range(total, world, k) for k in range(world))]
    flat = shard.unpack_bits(out.numpy(), sizes)
    q.put((rank, np.nonzero(flat)[0].tolist()))
    dist.destroy_process_group()


@pytest.mark.parametrize("total", [1001, 64])
def test_allgather_verdicts_gloo_world2(total):
    world = 2
    bad = [0, 5, total // 2, total - 1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, total, bad, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(world))
    for p in ps:
        p.join(timeout=60)
    assert res[0] == res[1] == sorted(set(bad))


def _recover_outputs(total, k):
    """Deterministic stand-ins for one Recover batch's outputs over `total` rounds (what dg_recover writes)."""
    rng = np.random.default_rng(total * 131 + k)
    sigs = rng.integers(0, 256, size=(total, 96), dtype=np.uint8)
    rs = (rng.random(total) < 0.05).astype(np.uint8) * 5
    ss = rng.choice(np.array([0, 1, 2, 255], np.uint8), size=(total, k))
    return sigs, rs, ss


def _rows_worker(rank, world, port, total, k, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    sigs, rs, ss = _recover_outputs(total, k)
    a, b = shard.round_range(total, world, rank)
    got = [shard.allgather_rows(torch.from_numpy(np.ascontiguousarray(x[a:b])), world, total).numpy()
           for x in (sigs, rs, ss)]
    q.put((rank, [g.tobytes() for g in got]))
    dist.destroy_process_group()


@pytest.mark.parametrize("total,k", [(1001, 64), (7, 256)])
def test_allgather_recover_outputs_gloo_world2(total, k):
    """Recover's outputs (96 B signatures, round statuses, per-share statuses), each rank holding its
    contiguous round range, all-gather to exactly the 1-rank arrays on every rank."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_rows_worker, args=(r, world, port, total, k, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(world))
    for p in ps:
        p.join(timeout=60)
    sigs, rs, ss = _recover_outputs(total, k)
    want = [sigs.tobytes(), rs.tobytes(), ss.tobytes()]
    assert res[0] == want and res[1] == want


def test_allgather_rows_world1_is_identity():
    x = torch.arange(30, dtype=torch.uint8).view(10, 3)
    assert torch.equal(shard.allgather_rows(x, 1, 10), x)
