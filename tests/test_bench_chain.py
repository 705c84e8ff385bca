"""bench.py's chain guard (round-3 verdict item 1): a configs[1] / configs[3] line measures the digest-pinned linked
chain (data/chain_v1_<n>.bin, made by the CPU twin) or nothing -- without a file that covers the rounds, or with a
file that fails its pinned SHA-256, the bench exits with status 3 instead of verifying unlinked rounds signed by the
library under test.  CPU only: the guard runs before anything touches the GPU."""
import os
import subprocess
import sys

import numpy as np
import pytest

import bench
from tools import synthetic as S

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_missing_chain_exits_3(tmp_path):
    with pytest.raises(SystemExit) as e:
        bench.require_chain(1000000, False, data_dir=str(tmp_path))
    assert e.value.code == 3
    assert bench.require_chain(1000000, True, data_dir=str(tmp_path)) is None


def test_tampered_chain_is_refused(tmp_path):
    p = tmp_path / "chain_v1_100000.bin"
    np.zeros((100000, 96), np.uint8).tofile(p)
    with pytest.raises(S.ChainFileError):
        S.find_chain(1000, str(tmp_path))
    with pytest.raises(SystemExit):
        bench.require_chain(1000, False, data_dir=str(tmp_path))


def test_bench_refuses_uncovered_rounds_at_n2():
    """`bench.py --gpus 2` run as a rank (WORLD_SIZE=2) asking for more rounds than any pinned chain holds exits 3
    before it imports torch or touches a GPU."""
    env = dict(os.environ, WORLD_SIZE="2", RANK="1", LOCAL_RANK="1")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--global-rounds", "2000000"],
                       env=env, capture_output=True, text=True, timeout=120, cwd=ROOT)
    assert r.returncode == 3, (r.returncode, r.stderr[-2000:])
    assert "refusing" in r.stderr


@pytest.mark.parametrize("n", sorted(S.CHAIN_SHA256))
def test_pinned_chain_files_match(n):
    """The chain files shipped with the tree match their digests (and so the configs[3] line and
    test_sharded_1m_chain_equals_one_batch run on the real linked chain)."""
    p = S.chain_path(n)
    if not os.path.exists(p):
        pytest.skip("data/chain_v1_%d.bin not generated in this checkout" % n)
    assert S.find_chain(n) == (n, p)


@pytest.mark.parametrize("world", [1, 2, 4, 8])
def test_every_rank_runs_the_one_batch_step(world):
    """BASELINE configs[3] at N = world (the 1M chain split N ways; configs[1] at N = 1): every rank's range is one
    device batch, and its verdicts are packed and all-gathered on the batch's own stream (bench.py
    consume_on_batch_stream: no side-stream wait) -- the N = 1 arrangement on every rank at world 2, 4, 8."""
    from drand_amd import shard

    G = 100000 if world == 1 else 1000000
    for rank in range(world):
        a, b = shard.round_range(G, world, rank)
        bounds = bench.batch_bounds(b - a)
        assert bounds == [(0, b - a)], (world, rank)
        assert bench.consume_on_batch_stream(len(bounds))
    # an explicit smaller --batch, or the blocking entry point, takes the side stream
    assert len(bench.batch_bounds(125000, 50000)) == 3 and not bench.consume_on_batch_stream(3)
    assert not bench.consume_on_batch_stream(1, use_sync=True)
    assert bench.batch_bounds(1000000) == [(0, 500000), (500000, 1000000)]
