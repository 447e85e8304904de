#!/usr/bin/env python3
"""Where the fused MT draw + split (make_shares_vec's default) stands against
the HBM: on the same share blocks (memory.share_block, 2 MiB chunks, and one
torch.empty block), per block

  * ceiling: dn_diag_tile_stream over the fused form's own bytes (8 B secret
    read + 5 x 66 B shares written per element), fastest grid;
  * range pattern: dn_diag_group_stream mode 0 — one 64-thread workgroup per
    contiguous 8192-element range (the generation kernel's substream), one
    quarter-tile per group (its wave-to-element mapping), no arithmetic;
  * tile pattern: mode 1 — 4 waves per 256-element tile (split_kernel's);
  * fused: make_shares_vec into the block (HIP events around the call, best
    of 5; under rocprof the generation kernel's own time is in the trace).

Prints one JSON line per block."""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "delta-node_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from bench import stream_ceiling  # noqa: E402
from delta_node.crypto import shamir  # noqa: E402
from delta_node.crypto.shamir import field, memory  # noqa: E402

N = 1 << int(os.environ.get("LOG2N", "24"))
dev = torch.device("cuda", 0)
torch.cuda.set_device(0)
vb = field.vec_bytes(N)
diag = ctypes.CDLL(os.path.join(ROOT, "delta-node_amd", "lib", "libdn_diag.so"))
vp = ctypes.c_void_p
stream = torch.cuda.current_stream()
sec = torch.randint(-(1 << 62), 1 << 62, (N,), dtype=torch.int64, device=dev)
gb = N * (8 + 5 * 66) / 1e9


def timed(fn, reps=5):
    fn()
    best = None
    for _ in range(reps):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record(stream)
        fn()
        e.record(stream)
        torch.cuda.synchronize()
        ms = s.elapsed_time(e)
        best = ms if best is None else min(best, ms)
    return best


def group(blk, mode, epw=8192, grid=0, nt=1):
    def f():
        rc = diag.dn_diag_group_stream(vp(sec.data_ptr()), vp(blk.data_ptr()), ctypes.c_uint64(vb),
                                       ctypes.c_uint64(N), 5, mode, ctypes.c_uint64(epw), grid, nt,
                                       vp(stream.cuda_stream))
        if rc:
            raise RuntimeError(f"dn_diag_group_stream rc={rc}")
    return f


blocks = [("share_block", memory.share_block((5, vb), dev)) for _ in range(3)]
blocks.append(("torch.empty", torch.empty((5, vb), dtype=torch.uint8, device=dev)))
ss = shamir.SecretShare(3)
ss.random.seed(7)
for rnd in range(2):
    for i, (kind, blk) in enumerate(blocks):
        r = {"round": rnd, "block": i, "kind": kind, "N": N, "GB": gb}
        c = stream_ceiling([sec], [8 * 256], [blk[x] for x in range(5)], [66 * 256] * 5, N // 256)
        r["ceiling_ms"] = c["ms"]
        r["range_nt_ms"] = timed(group(blk, 0, nt=1))
        r["range_plain_ms"] = timed(group(blk, 0, nt=0))
        r["range_4096_nt_ms"] = timed(group(blk, 0, epw=4096, nt=1))
        r["tile_nt_ms"] = min(timed(group(blk, 1, grid=g, nt=1)) for g in (2048, 8192, 65536))
        r["fused_ms"] = timed(lambda: ss.make_shares_vec(sec, 5, out=blk))
        for k in ("ceiling_ms", "range_nt_ms", "range_plain_ms", "range_4096_nt_ms", "tile_nt_ms", "fused_ms"):
            r[k.replace("_ms", "_TBps")] = gb / r[k]
        print(json.dumps(r), flush=True)
