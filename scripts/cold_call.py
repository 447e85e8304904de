#!/usr/bin/env python3
"""The first make_shares_vec of a fresh process.

The reference's callers split once per round (runner/horizontal/agg.py:142-153),
so what a round pays is a process's FIRST call, not the warm rate.  Run in a
fresh process (bench.py starts it as a child); prints one JSON line.

  --mode e2e     secrets resident on the device (untimed), then the first
                 make_shares_vec(sec, 5) with out=None, wall time to return:
                 share-block mapping + probe, the MT jump rows and job tables,
                 their upload, the draw + split.  Then the same call again
                 after the first output is dropped (the pool's idle block).
  --force-miss   every share-block probe try misses the keep bar (the
                 class's best rate set unreachable, PROBE_FAST likewise): the
                 worst first call, tries bounded by memory.PROBE_TIME_BUDGET.
  --mode phases  the same costs one at a time: the share block alone
                 (memory.share_block: chunk mapping + write-rate probe), a
                 first 2^12 call (kernels, scratch), then the first 2^N call
                 into the block (the 2^N shape's rows and job tables), then a
                 second one.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "delta-node_amd"))


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--log2n", type=int, default=24)
    ap.add_argument("--mode", choices=("e2e", "phases"), default="e2e")
    ap.add_argument("--force-miss", action="store_true")
    args = ap.parse_args()
    t_start = time.perf_counter()
    import numpy as np
    import torch

    t_torch = time.perf_counter()
    from delta_node.crypto import shamir
    from delta_node.crypto.shamir import _native, field, memory

    _native.lib()
    t_lib = time.perf_counter()
    torch.cuda.init()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    n = 1 << args.log2n
    sec = torch.from_numpy(np.random.default_rng(5).integers(-(1 << 63), (1 << 63) - 1, n, dtype=np.int64,
                                                            endpoint=True)).to(dev)
    torch.cuda.synchronize()
    t_ready = time.perf_counter()
    out = {"mode": args.mode, "N": n, "import_torch_s": t_torch - t_start, "load_lib_s": t_lib - t_torch,
           "cuda_init_and_upload_s": t_ready - t_lib}

    def timed(fn):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        r = fn()
        torch.cuda.synchronize()
        return r, (time.perf_counter() - t0) * 1e3

    if args.force_miss:
        memory.PROBE_FAST = float("inf")
        kind = (0, 5, (5 * field.vec_bytes(n)).bit_length())  # the share block's class (memory._alloc_probed)
        memory._best_rate[kind] = float("inf")
    ss = shamir.SecretShare(3)
    ss.random.seed(9)
    if args.mode == "e2e":
        sh, out["first_ms"] = timed(lambda: ss.make_shares_vec(sec, 5))
        out["pool_after_first"] = memory.pool_stats()
        del sh
        sh, out["second_ms"] = timed(lambda: ss.make_shares_vec(sec, 5))
        out["pool_after_second"] = memory.pool_stats()
    else:
        blk, out["share_block_ms"] = timed(lambda: memory.share_block((5, field.vec_bytes(n)), dev))
        out["pool_after_block"] = memory.pool_stats()
        small = torch.empty((5, field.vec_bytes(4096)), dtype=torch.uint8, device=dev)
        _, out["first_2e12_ms"] = timed(lambda: ss.make_shares_vec(sec[:4096], 5, out=small))
        _, out["first_into_block_ms"] = timed(lambda: ss.make_shares_vec(sec, 5, out=blk))
        _, out["second_into_block_ms"] = timed(lambda: ss.make_shares_vec(sec, 5, out=blk))
    print(json.dumps(out), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
