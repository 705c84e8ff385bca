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
