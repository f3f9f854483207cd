"""bench.py's node batches: every rank builds its shard_range slice of ONE node batch (items are functions of the seed
and the global index), and the node-wide expected bitmaps it checks after the RCCL all-gather are the union of the
slices.  CPU-only: a stand-in engine returns placeholder bytes for keys and signatures (the GPU tests and the bench
itself check real verdicts); what is tested here is the slicing and the bookkeeping of corrupted positions."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import bench
from charon_amd.shard import gather_bitmap_rows, shard_range, unpack_bitmap


class FakeImpl:
    def secret_to_public_key_batch(self, sks):
        return [b"P" + s[:47] for s in sks], [0] * len(sks)

    def sign_batch(self, sks, msgs):
        return [(s + m + bytes(96))[:96] for s, m in zip(sks, msgs)], [0] * len(sks)


@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_c2_slices_tile_the_node_batch(world):
    impl = FakeImpl()
    keys = bench.share_keys(impl, 64, "c2")
    n_node = 3000
    roots, bad = [], set()
    for r in range(world):
        lo, hi = shard_range(n_node, r, world)
        _, rts, _, b = bench.make_c2(impl, keys, lo, hi)
        roots += rts
        bad |= {lo + i for i in b}
    whole = bench.make_c2(impl, keys, 0, n_node)
    assert roots == whole[1]
    assert bad == whole[3] == {i for i in range(n_node) if bench.c2_is_bad(i)[0]}
    assert 5 <= len(bad) <= 60  # ~1%


@pytest.mark.parametrize("world,n_roots", [(1, 0), (2, 0), (3, 0), (2, 5), (8, 3)])
def test_c4_slices_tile_the_node_batch(world, n_roots):
    impl = FakeImpl()
    keys = bench.share_keys(impl, 32, "c4")
    V = 1001
    msgs, bad, pks = [], set(), []
    for r in range(world):
        lo, hi = shard_range(V, r, world)
        p, s, midx, rts, b = bench.make_c4(impl, keys, "c4i", lo, hi, V, n_roots)
        assert len(p) == len(s) == len(midx) == 4 * (hi - lo)
        msgs += [rts[m] for m in midx]
        bad |= {4 * lo + i for i in b}
        pks += p
    whole = bench.make_c4(impl, keys, "c4i", 0, V, V, n_roots)
    assert msgs == [whole[3][m] for m in whole[2]]  # every item signs the same root in the slice and in the whole
    assert pks == whole[0]
    assert bad == whole[4] == bench.c4_node_bad("c4i", V, 32)
    if n_roots:
        assert len(set(msgs)) == n_roots
    else:
        assert len(set(msgs)) == V


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        # C5-shaped rows: a C4 slice plus a proposer slice, lengths differ across ranks
        rows_len = [4 * (shard_range(1001, r, world)[1] - shard_range(1001, r, world)[0])
                    + 4 * (shard_range(32, r, world)[1] - shard_range(32, r, world)[0]) for r in range(world)]
        g = torch.Generator().manual_seed(100 + rank)
        local = torch.randint(0, 3, (rows_len[rank],), generator=g, dtype=torch.int32)
        rows = gather_bitmap_rows(local, max(rows_len))
        ok = True
        for r in range(world):
            gr = torch.Generator().manual_seed(100 + r)
            want = torch.randint(0, 3, (rows_len[r],), generator=gr, dtype=torch.int32) == 0
            ok &= bool(torch.equal(unpack_bitmap(rows[r], rows_len[r]), want))
        q.put((rank, ok))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_gloo_uneven_row_gather(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
    res = [q.get(timeout=10) for _ in range(world)]
    assert all(ok for _, ok in res), res
