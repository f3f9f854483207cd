"""Multi-GPU sharding of the verify / aggregate batches.

One process per GPU.  Validators are split into contiguous index ranges (shard_range), so all partials
of one distributed validator land on one GPU and ThresholdAggregate needs no exchange.  The only
collectives are all-gathers of results: the per-rank verify bitmaps (1 bit per item; RLC bitmaps
too) and the 96-byte aggregate signatures -- over RCCL/xGMI (backend "nccl") on MI355X nodes, over
gloo in the CPU tests.  There is no all-reduce on the data path.  Shards differ in size by at most one
item, so every rank pads its block to the largest shard before the all-gather and the receiver cuts
each row back to that rank's shard_range.
"""
from __future__ import annotations

from typing import Tuple

import torch
import torch.distributed as dist


def shard_range(n_items: int, rank: int, world: int) -> Tuple[int, int]:
    """Contiguous [lo, hi) slice of n_items owned by `rank` (sizes differ by at most 1)."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError("bad rank/world")
    base, extra = divmod(n_items, world)
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


_WEIGHTS = {}


def pack_bitmap(status: torch.Tensor) -> torch.Tensor:
    """int32 status[n] (0 = verified) -> uint8 bitmap[ceil(n/8)], bit i%8 of byte i/8 = item i ok.
    Runs on the status tensor's device (no host round trip)."""
    n = status.numel()
    ok = (status == 0).to(torch.uint8)
    pad = (-n) % 8
    if pad:
        ok = torch.cat([ok, torch.zeros(pad, dtype=torch.uint8, device=ok.device)])
    key = ok.device
    w = _WEIGHTS.get(key)
    if w is None:
        w = _WEIGHTS[key] = (2 ** torch.arange(8, device=ok.device)).to(torch.uint8)
    return (ok.view(-1, 8) * w).sum(dim=1, dtype=torch.uint8)


def unpack_bitmap(bits: torch.Tensor, n: int) -> torch.Tensor:
    """Inverse of pack_bitmap: bool[n]."""
    shifts = torch.arange(8, device=bits.device)
    return ((bits.view(-1, 1).to(torch.int32) >> shifts) & 1).view(-1)[:n].bool()


def _max_shard(n_items: int, world: int) -> int:
    return (n_items + world - 1) // world


def _gather_padded(local: torch.Tensor, width: int, group=None) -> torch.Tensor:
    """All-gather one uint8 block per rank, each zero-padded to `width` bytes -> [world, width]."""
    world = dist.get_world_size(group)
    if local.numel() > width:
        raise ValueError("local block larger than the padded width")
    # gloo has no device-tensor all-gather: a gloo group (the CPU tests, or a multi-rank rehearsal on one GPU) stages
    # through host memory; RCCL ("nccl") gathers device tensors over xGMI directly
    stage = local.is_cuda and dist.get_backend(group) == "gloo"
    dev = torch.device("cpu") if stage else local.device
    buf = torch.zeros(width, dtype=torch.uint8, device=dev)
    buf[:local.numel()] = local.reshape(-1).to(dev)
    out = torch.empty(world * width, dtype=torch.uint8, device=dev)
    dist.all_gather_into_tensor(out, buf, group=group)
    return out.view(world, width).to(local.device)


def gather_bitmaps(local_bits: torch.Tensor, n_items: int = None, group=None) -> torch.Tensor:
    """All-gather per-rank bitmaps -> [world, nbytes] on every rank.  With n_items (the node batch) every
    row is padded to the largest shard's ceil(size/8) bytes, so uneven shards gather too."""
    world = dist.get_world_size(group)
    width = local_bits.numel() if n_items is None else (_max_shard(n_items, world) + 7) // 8
    return _gather_padded(local_bits, width, group)


def gather_bitmap_rows(local_status: torch.Tensor, max_items: int, group=None) -> torch.Tensor:
    """All-gather per-rank status vectors of different lengths (at most max_items each) as packed ok-bitmaps:
    [world, ceil(max_items / 8)] on every rank; row r holds rank r's items in its first bits."""
    return _gather_padded(pack_bitmap(local_status), (max_items + 7) // 8, group)


def gather_node_bitmap(local_status: torch.Tensor, n_items: int, group=None) -> torch.Tensor:
    """Per-rank status of shard_range(n_items, rank, world) -> bool[n_items] ok-bitmap of the whole node batch."""
    world = dist.get_world_size(group)
    rows = gather_bitmaps(pack_bitmap(local_status), n_items, group)
    parts = []
    for r in range(world):
        lo, hi = shard_range(n_items, r, world)
        parts.append(unpack_bitmap(rows[r], hi - lo))
    return torch.cat(parts)


def gather_aggregates(local_sigs: torch.Tensor, n_groups: int, group=None) -> torch.Tensor:
    """Per-rank aggregate signatures (uint8, 96 bytes per validator of shard_range(n_groups, rank, world)) ->
    uint8[n_groups * 96] in validator order on every rank."""
    world = dist.get_world_size(group)
    rows = _gather_padded(local_sigs, 96 * _max_shard(n_groups, world), group)
    parts = []
    for r in range(world):
        lo, hi = shard_range(n_groups, r, world)
        parts.append(rows[r, :96 * (hi - lo)])
    return torch.cat(parts)
