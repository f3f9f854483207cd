"""World-size-2 gloo tests of the multi-GPU path (charon_amd/shard.py) on CPU: contiguous
validator-index shards and the bitmap all-gather the bench performs over RCCL on MI355X nodes."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from charon_amd.shard import (gather_aggregates, gather_bitmaps, gather_node_bitmap, pack_bitmap, shard_range,
                              unpack_bitmap)


def test_shard_range_partitions():
    for n in (0, 1, 7, 1000, 1 << 20):
        for world in (1, 2, 3, 8):
            spans = [shard_range(n, r, world) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
            sizes = [hi - lo for lo, hi in spans]
            assert max(sizes) - min(sizes) <= 1


def test_pack_unpack_roundtrip():
    g = torch.Generator().manual_seed(3)
    for n in (1, 8, 13, 4096, 65537):
        st = torch.randint(0, 4, (n,), generator=g, dtype=torch.int32)
        bits = pack_bitmap(st)
        assert bits.numel() == (n + 7) // 8
        assert torch.equal(unpack_bitmap(bits, n), st == 0)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n_items, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        # every rank derives the same global status vector, verifies only its shard
        g = torch.Generator().manual_seed(11)
        full = torch.randint(0, 4, (n_items,), generator=g, dtype=torch.int32)
        lo, hi = shard_range(n_items, rank, world)
        local = full[lo:hi]
        bits = gather_bitmaps(pack_bitmap(local), n_items)
        got = torch.cat([unpack_bitmap(bits[r], shard_range(n_items, r, world)[1] - shard_range(n_items, r, world)[0])
                         for r in range(world)])
        q.put((rank, bool(torch.equal(got, full == 0))))
        q.put((rank, bool(torch.equal(gather_node_bitmap(local, n_items), full == 0))))
        # aggregate signatures: each rank owns a contiguous validator range (uneven when n_groups % world != 0)
        n_groups = n_items // 3 + 1
        allsig = torch.randint(0, 256, (n_groups * 96,), generator=g, dtype=torch.uint8)
        glo, ghi = shard_range(n_groups, rank, world)
        q.put((rank, bool(torch.equal(gather_aggregates(allsig[96 * glo:96 * ghi], n_groups), allsig))))
        # max-over-ranks timing reduce used by bench.py
        t = torch.tensor([float(rank + 1)], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        q.put((rank, float(t.item()) == float(world)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,n_items", [(2, 4096 * 2), (2, 4097 * 2 + 1), (3, 1001)])
def test_gloo_bitmap_gather(world, n_items):
    """Equal shards (the weak-scaling bench) and uneven ones (a node batch that does not divide by world)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n_items, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
        assert p.exitcode == 0
    results = [q.get(timeout=5) for _ in range(4 * world)]
    assert all(ok for _, ok in results), results
