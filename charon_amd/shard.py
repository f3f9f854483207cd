"""Multi-GPU sharding of the verify / aggregate batches.

One process per GPU.  Validators are split into contiguous index ranges, so all partials of one
distributed validator land on one GPU and ThresholdAggregate needs no exchange.  The only
collective is one all-gather of the per-rank verify bitmaps (1 bit per item) -- over RCCL/xGMI
(backend "nccl") on MI355X nodes, over gloo in the CPU tests.  There is no all-reduce on the data
path.
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


def gather_bitmaps(local_bits: torch.Tensor, group=None) -> torch.Tensor:
    """All-gather equal-sized per-rank bitmaps -> [world, nbytes] on every rank."""
    world = dist.get_world_size(group)
    out = torch.empty(world * local_bits.numel(), dtype=local_bits.dtype, device=local_bits.device)
    dist.all_gather_into_tensor(out, local_bits.contiguous(), group=group)
    return out.view(world, -1)
