#!/usr/bin/env python3
"""make_shares_vec (the fused bit-exact MT draw + split, 3-of-5) under one
library (DN_SHAMIR_LIB selects it): at 2^24 on three share blocks
(memory.share_block) and one torch.empty block, HIP events around each call,
best of 5 per block; wall time per call at 2^20 / 2^16 / 2^12 (50 calls).
Checks the output against draw-then-split once per size.  One JSON line."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "delta-node_amd"))

import torch  # noqa: E402

from delta_node.crypto import shamir  # noqa: E402
from delta_node.crypto.shamir import _native, field, memory  # noqa: E402

dev = torch.device("cuda", 0)
torch.cuda.set_device(0)
stream = torch.cuda.current_stream()
res = {"lib": os.path.basename(_native.lib_path())}
N = 1 << 24
vb = field.vec_bytes(N)
sec = torch.randint(-(1 << 62), 1 << 62, (N,), dtype=torch.int64, device=dev)
blocks = [memory.share_block((5, vb), dev) for _ in range(3)]
blocks.append(torch.empty((5, vb), dtype=torch.uint8, device=dev))
ss = shamir.SecretShare(3)
ss.random.seed(9)
ms = []
for blk in blocks:
    for _ in range(2):
        ss.make_shares_vec(sec, 5, out=blk)
    best = None
    for _ in range(5):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record(stream)
        ss.make_shares_vec(sec, 5, out=blk)
        e.record(stream)
        torch.cuda.synchronize()
        t = s.elapsed_time(e)
        best = t if best is None else min(best, t)
    ms.append(best)
res["2^24_ms_by_block"] = ms
res["2^24_ms_share_block_median"] = sorted(ms[:3])[1]
ok = {}
for lg in (24, 20, 16, 12):
    n = 1 << lg
    a, b = shamir.SecretShare(3), shamir.SecretShare(3)
    a.random.seed(lg)
    b.random.seed(lg)
    x = sec[:n]
    out = a.make_shares_vec(x, 5)
    co = b.draw_coeffs_vec(n, dev)
    ref = torch.empty_like(out)
    _native.split_u64(x, co, ref, n, 3, 5)
    ok[f"2^{lg}"] = bool(torch.equal(out, ref)) and a.random.getstate() == b.random.getstate()
    if lg < 24:
        sh = torch.empty((5, field.vec_bytes(n)), dtype=torch.uint8, device=dev)
        for _ in range(5):
            a.make_shares_vec(x, 5, out=sh)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(50):
            a.make_shares_vec(x, 5, out=sh)
        torch.cuda.synchronize()
        res[f"2^{lg}_ms_per_call"] = (time.perf_counter() - t0) / 50 * 1e3
res["equal_draw_then_split"] = ok
print(json.dumps(res))
