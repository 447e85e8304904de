"""Element sharding of the vector path across the GPUs of one node.

One process per GPU (torch.distributed, backend "nccl" = RCCL over xGMI).
Every element is independent, so the split needs no collective: rank r owns
the contiguous, tile-aligned element range `shard_range(N, r, world)` and
splits it locally.  Because the M521 layout is tiled (256 elements per
16896-byte tile), a tile-aligned shard of a vector is a contiguous byte range
of the full vector, so the one exchange step — every rank receiving every
share vector — is one all-gather per share row straight into that row of the
full vectors.

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


def _via_host(t, group) -> bool:
    """gloo is a host transport: device tensors are gathered through host
    memory (the multi-rank GPU tests run every rank on one GPU with gloo; the
    product backend is nccl = RCCL, which moves device memory directly)."""
    import torch.distributed as dist

    return t.is_cuda and dist.get_backend(group) == "gloo"


def allgather_share_blocks(local_block, n_total: int, group=None):
    """Gather every rank's share block into full share vectors on every rank.

    local_block  uint8 [S, shard_tiles(n_total, world) * TILE_BYTES] (this rank's
                 shard, padded to the common tile count)
    Returns uint8 [S, world * shard_bytes]; its first vec_bytes(n_total) bytes
    per row are the full tiled vectors (the rest is tile padding).

    One all-gather per share row, straight into that row of the output: rank
    r's shard lands at byte r * shard_bytes, which is where its tiles belong
    in the full vector, so no permute copy follows and the output is the only
    buffer (S calls of world * shard_bytes each — 9 x 4.4 GB at config 4 —
    are far past the size where RCCL's per-call cost matters).
    """
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    S, B = local_block.shape
    if B != shard_tiles(n_total, world) * field.TILE_BYTES:
        raise ValueError("allgather_share_blocks: block is not padded to the common shard size")
    host = _via_host(local_block, group)
    src = local_block.cpu() if host else local_block.contiguous()
    out = torch.empty((S, world * B), dtype=local_block.dtype, device=src.device)
    for s in range(S):
        dist.all_gather_into_tensor(out[s], src[s], group=group)
    return out.to(local_block.device) if host else out


def draw_coeffs_sharded(ss, n_total: int, device=None, group=None):
    """This rank's slice of the coefficients `ss.draw_coeffs_vec(n_total)`
    would draw — the reference's MT19937 stream (shamir.py:59-61), bit-exact —
    without any rank drawing the others' words: each rank jumps to its shard's
    first word (dn_mt19937_skip) and draws only its tiles; every rank's
    `ss.random` ends as after the whole draw.  A rejected 521-bit draw in any
    shard (odds ~2^-520 each) shifts the later shards: the ranks agree on it
    (one all-reduce of a flag) and then each redraws the whole stream on the
    host and keeps its slice, so the result is exact either way.

    Returns uint8 [t-1, shard_tiles(n_total, world) * TILE_BYTES] (padded like
    `allgather_share_blocks` expects; the elements are shard_range's)."""
    import random

    import torch
    import torch.distributed as dist

    world, rank = dist.get_world_size(group), dist.get_rank(group)
    lo, hi = shard_range(n_total, rank, world)
    tm1 = max(ss.threshold, 1) - 1
    B = shard_tiles(n_total, world) * field.TILE_BYTES
    state0 = ss.random.getstate()
    out = torch.zeros((tm1, B), dtype=torch.uint8, device=device)
    if hi > lo and tm1 > 0:
        blk = ss.draw_coeffs_vec(hi - lo, device, elem_offset=lo, n_total=n_total)
        out[:, : blk.shape[1]].copy_(blk)
        rejected = ss.last_draw_rejected
    else:
        from . import _native

        _native.mt_skip(ss.random, 17 * tm1 * n_total)
        rejected = False
    flag = torch.tensor([int(rejected)], dtype=torch.int32, device=out.device)
    if _via_host(flag, group):
        flag = flag.cpu()
    dist.all_reduce(flag, op=dist.ReduceOp.MAX, group=group)
    if int(flag.item()):
        from . import _native

        rng = random.Random()
        rng.setstate(state0)
        full = _native.mt_draw_coeffs(rng, n_total, tm1)  # every word, in order: exact with rejections
        ss.random.setstate(rng.getstate())
        t0 = lo // field.TILE
        nb = field.vec_bytes(hi - lo) if hi > lo else 0
        out.zero_()
        if nb:
            out[:, :nb].copy_(torch.from_numpy(full[:, t0 * field.TILE_BYTES: t0 * field.TILE_BYTES + nb]))
    return out
