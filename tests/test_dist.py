"""Multi-process element sharding (CPU, gloo, world_size 2 and 3).

Each rank computes the shares of its tile-aligned shard (here, on a CPU-only
host, with the C oracle standing in for the per-rank kernel), packs them into
its padded block and all-gathers; the gathered vectors must equal the
unsharded split byte for byte.  This is the data path `bench.py` and BASELINE
config 4 use over RCCL.  The same path with the HIP kernels — device MT
draw per shard, HIP split, gather, reconstruct — runs in tests/test_gpu_dist.py
(fresh child ranks on one GPU, gloo).
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from delta_node.crypto.shamir import dist as sdist
from delta_node.crypto.shamir import field


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, N, t, n, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for p in (os.path.join(root, "delta-node_amd"), root, os.path.join(root, "tests")):
        if p not in sys.path:
            sys.path.insert(0, p)
    from oracle import c_oracle
    from golden.fixtures import secrets_int64

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        sec = secrets_int64(3, N)
        co = c_oracle.draw_coeffs(3, N, t - 1)
        lo, hi = sdist.shard_range(N, rank, world)
        B = sdist.shard_tiles(N, world) * field.TILE_BYTES
        block = np.zeros((n, B), dtype=np.uint8)
        if hi > lo:
            sh = c_oracle.split(sec[lo:hi], co[lo:hi], t, n)  # [n, hi-lo, 17]
            for x in range(n):
                v = field.limbs_to_vec(sh[x])
                block[x, : v.size] = v
        full = sdist.allgather_share_blocks(torch.from_numpy(block), N)
        if rank == 0:
            want = c_oracle.split(sec, co, t, n)
            ok = all(np.array_equal(full[x, : field.vec_bytes(N)].numpy(), field.limbs_to_vec(want[x]))
                     for x in range(n))
            q.put(ok)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,N", [(2, 1000), (2, 512), (3, 1001)])
def test_sharded_split_allgather_equals_unsharded(world, N):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, N, 3, 5, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
    assert all(p.exitcode == 0 for p in procs)
    assert q.get(timeout=10) is True


def test_shard_ranges_cover_exactly():
    for N in (0, 1, 255, 256, 1000, 1 << 20):
        for world in (1, 2, 3, 8):
            ranges = [sdist.shard_range(N, r, world) for r in range(world)]
            assert ranges[0][0] == 0 and ranges[-1][1] == N
            for (a, b), (c, d) in zip(ranges, ranges[1:]):
                assert b == c and (a % field.TILE == 0 or a == N)
            assert all(hi - lo <= sdist.shard_tiles(N, world) * field.TILE for lo, hi in ranges)


def _allreduce_worker(rank, world, port, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "delta-node_amd"))
    from delta_node.utils.agg import allreduce_sum

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        rng = np.random.default_rng(rank)
        part = torch.from_numpy(rng.integers(-2**63, 2**63 - 1, 1000, dtype=np.int64, endpoint=True))
        mine = part.clone()
        allreduce_sum(part)
        parts = [torch.from_numpy(np.random.default_rng(r).integers(-2**63, 2**63 - 1, 1000, dtype=np.int64,
                                                                    endpoint=True)) for r in range(world)]
        want = parts[0].clone()
        for p in parts[1:]:
            want += p  # int64 wrap, as numpy's += in make_masked_results
        if rank == 0:
            q.put(bool(torch.equal(part, want)) and not torch.equal(mine, want))
    finally:
        dist.destroy_process_group()


def test_allreduce_masked_partial_sums_wrap_like_numpy():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_allreduce_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
    assert all(p.exitcode == 0 for p in procs)
    assert q.get(timeout=10) is True


def _mt_shard_worker(rank, world, port, N, t, q):
    import random
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "delta-node_amd"))
    from delta_node.crypto import shamir
    from delta_node.crypto.shamir import _native
    from delta_node.crypto.shamir import dist as sd

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        ss = shamir.SecretShare(t)
        ss.random.seed(4242)
        ss.random.getrandbits(32 * 77)  # start mid-array
        start = ss.random.getstate()
        blk = sd.draw_coeffs_sharded(ss, N, device="cpu")
        full = sd.allgather_share_blocks(blk, N)
        ref = random.Random()
        ref.setstate(start)
        want = _native.mt_draw_coeffs(ref, N, t - 1)  # the whole stream on one host, in order
        ok = np.array_equal(full[:, : want.shape[1]].numpy(), want) and ss.random.getstate() == ref.getstate()
        q.put((rank, bool(ok)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,N,t", [(2, 1000, 3), (3, 70001, 3), (2, 40000, 5)])
def test_sharded_mt_draw_equals_one_stream(world, N, t):
    """dist.draw_coeffs_sharded: every rank jumps to its shard of the
    reference's MT19937 coefficient stream and draws only that; the gathered
    blocks equal one sequential draw and every rank's random.Random ends in the
    sequential draw's state (host draw path; the device path is the gpu tests')."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_mt_shard_worker, args=(r, world, port, N, t, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(180)
    assert all(p.exitcode == 0 for p in procs)
    res = [q.get(timeout=10) for _ in range(world)]
    assert all(ok for _, ok in res), res
