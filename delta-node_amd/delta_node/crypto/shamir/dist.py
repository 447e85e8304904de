"""Element sharding of the vector path across the GPUs of one node.

One process per GPU (torch.distributed, backend "nccl" = RCCL over xGMI).
Every element is independent, so the split needs no collective: rank r owns
the contiguous, tile-aligned element range `shard_range(N, r, world)` and
splits it locally.  Because the M521 layout is tiled (256 elements per
16896-byte tile), a tile-aligned shard of a vector is a contiguous byte range
of the full vector, so the one exchange step — every rank receiving every
share vector — is a single all-gather of each rank's [n_shares, shard_bytes]
block followed by a [world, S, B] -> [S, world*B] permute.

Semantically, handing share x to party x is an all-to-all; the all-gather
(every rank gets all shares) is what BASELINE config 4 specifies and is
reported separately from split throughput.
"""
from __future__ import annotations

from typing import Tuple

from . import field


def shard_range(n_total: int, rank: int, world: int) -> Tuple[int, int]:
    """[lo, hi) elements of rank `rank`: equal whole-tile shards (the last may be short)."""
    tiles = (n_total + field.TILE - 1) // field.TILE
    per = (tiles + world - 1) // world
    lo = min(n_total, rank * per * field.TILE)
    hi = min(n_total, (rank + 1) * per * field.TILE)
    return lo, hi


def shard_tiles(n_total: int, world: int) -> int:
    """Tiles per rank (every rank's block is padded to this many tiles)."""
    tiles = (n_total + field.TILE - 1) // field.TILE
    return (tiles + world - 1) // world


def allgather_share_blocks(local_block, n_total: int, group=None):
    """Gather every rank's share block into full share vectors on every rank.

    local_block  uint8 [S, shard_tiles(n_total, world) * TILE_BYTES] (this rank's
                 shard, padded to the common tile count)
    Returns uint8 [S, world * shard_bytes]; its first vec_bytes(n_total) bytes
    per row are the full tiled vectors (the rest is tile padding).
    """
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    S, B = local_block.shape
    if B != shard_tiles(n_total, world) * field.TILE_BYTES:
        raise ValueError("allgather_share_blocks: block is not padded to the common shard size")
    gathered = torch.empty((world * S, B), dtype=local_block.dtype, device=local_block.device)
    dist.all_gather_into_tensor(gathered, local_block.contiguous(), group=group)
    return gathered.view(world, S, B).permute(1, 0, 2).reshape(S, world * B)
