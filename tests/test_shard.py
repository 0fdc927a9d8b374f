"""Multi-GPU path on CPU: row-group sharding and the max-over-ranks timing the
benchmark uses, run as a real world_size-2 torch.distributed job on gloo."""
import os
import socket

import pytest

from pqgpu import shard


@pytest.mark.parametrize("groups", [1, 2, 7, 16, 256])
@pytest.mark.parametrize("world", [1, 2, 4, 8])
def test_row_group_ranges_partition(groups, world):
    got = [shard.row_group_range(groups, r, world) for r in range(world)]
    assert got[0][0] == 0 and got[-1][1] == groups
    for (a0, a1), (b0, b1) in zip(got, got[1:]):
        assert a1 == b0 and a0 <= a1
    sizes = [b - a for a, b in got]
    assert max(sizes) - min(sizes) <= 1


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    g0, g1 = shard.row_group_range(16 * world, rank, world)
    t = shard.max_over_ranks(1.0 + rank, dist)
    q.put((rank, g0, g1, t))
    dist.barrier()
    dist.destroy_process_group()


def test_gloo_world2_shards_and_max():
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    out = sorted(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert [(g0, g1) for _, g0, g1, _ in out] == [(0, 16), (16, 32)]
    assert all(t == 2.0 for *_, t in out)
