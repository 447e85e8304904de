"""One rank of the multi-rank GPU test (tests/test_gpu_dist.py), run as a fresh
child process: BASELINE config 4's product path with the gloo backend, every
rank on cuda:0 (or, with DN_DIST_BACKEND=nccl, RCCL at world size 1) —

  dist.draw_coeffs_sharded (device MT19937 jump-ahead to the rank's shard of
  the reference's one coefficient stream) -> the HIP split (split_u64) of the
  rank's shard -> dist.allgather_share_blocks -> the reconstruct of the rank's
  shard from the gathered vectors.

    RANK=r WORLD_SIZE=w MASTER_ADDR=127.0.0.1 MASTER_PORT=p python gpu_dist_worker.py OUT.json N t n mt_seed sec_seed

Writes {rank, digest (rank 0: of the gathered block), state_equal, roundtrip,
block_equal_single} to OUT.json.<rank>.
"""
import json
import os
import random
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "delta-node_amd"), ROOT, os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def main():
    out_path, N, t, n, mt_seed, sec_seed = sys.argv[1], *map(int, sys.argv[2:7])
    from delta_node.crypto import shamir
    from delta_node.crypto.shamir import _native, field
    from delta_node.crypto.shamir import dist as sdist
    from golden.fixtures import chunk_digests, combine_digests, secrets_int64

    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    backend = os.environ.get("DN_DIST_BACKEND", "gloo")
    if backend == "nccl":  # RCCL: device tensors move GPU to GPU, no host staging
        dist.init_process_group("nccl", device_id=dev)
    else:
        dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    res = {"rank": rank, "world": world, "backend": dist.get_backend()}
    try:
        lo, hi = sdist.shard_range(N, rank, world)
        nl = hi - lo
        B = sdist.shard_tiles(N, world) * field.TILE_BYTES
        vb = field.vec_bytes(nl)
        sec_all = secrets_int64(sec_seed, N)
        sec = torch.from_numpy(sec_all[lo:hi].copy()).to(dev)
        ss = shamir.SecretShare(t)
        ss.random.seed(mt_seed)
        cb = sdist.draw_coeffs_sharded(ss, N, dev)  # [t-1, B] on the GPU
        res["device_draw"] = bool(cb.is_cuda) and not ss.last_draw_rejected
        block = torch.zeros((n, B), dtype=torch.uint8, device=dev)
        if nl:
            coeffs = cb[:, :vb].contiguous()
            shares = torch.empty((n, vb), dtype=torch.uint8, device=dev)
            _native.split_u64(sec, coeffs, shares, nl, t, n)
            block[:, :vb].copy_(shares)
        res["via_host"] = sdist._via_host(block, None)
        full = sdist.allgather_share_blocks(block, N)  # [n, world * B] on every rank
        res["gathered_on_device"] = bool(full.is_cuda)
        torch.cuda.synchronize()
        fv = full[:, : field.vec_bytes(N)]
        # every rank's random.Random as after ONE sequential draw of the whole stream
        ref = random.Random(mt_seed)
        _native.mt_draw_coeffs(ref, N, t - 1)
        res["state_equal"] = ss.random.getstate() == ref.getstate()
        # reconstruct this rank's shard from the GATHERED vectors (shares 1, 3, 5, ...)
        xs = list(range(1, n + 1, 2))[: max(t, 1)] if n >= 2 * t - 1 else list(range(1, t + 1))
        ok = True
        if nl:
            t0 = lo // field.TILE
            rows = [fv[x - 1, t0 * field.TILE_BYTES: t0 * field.TILE_BYTES + vb].contiguous() for x in xs]
            rec = torch.empty(nl, dtype=torch.int64, device=dev)
            _native.reconstruct(rows, _native.lagrange(xs, t), out_u64=rec, n=nl)
            ok = bool(torch.equal(rec, sec))
        res["roundtrip"] = ok
        res["xs"] = xs
        if rank == 0:
            h = fv.cpu().numpy()
            planes = np.stack([field.vec_to_planes(h[s], N) for s in range(n)])
            res["digest"] = combine_digests(chunk_digests(planes))
            # the unsharded single-process split of the same vector, same stream
            ss1 = shamir.SecretShare(t)
            ss1.random.seed(mt_seed)
            one = ss1.make_shares_vec(torch.from_numpy(sec_all), n)
            res["block_equal_single"] = bool(torch.equal(one, fv))
    finally:
        dist.destroy_process_group()
    with open(f"{out_path}.{rank}", "w") as f:
        json.dump(res, f)


if __name__ == "__main__":
    main()
