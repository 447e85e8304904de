#!/usr/bin/env python3
"""Rate of the bit-exact MT19937 coefficient draw (the reference's
self.random.randint(1, p-1) stream, shamir.py:59-61) for 2^24 elements,
t = 3: host C++ draw + H2D vs the device draw (jump-ahead substreams).
Prints one JSON object."""
import json
import os
import random
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "delta-node_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from delta_node.crypto.shamir import _native, field  # noqa: E402

N, TM1 = 1 << int(os.environ.get("LOG2N", "24")), 2
dev = torch.device("cuda", 0)
out = {"N": N, "tm1": TM1, "words": 17 * N * TM1}
blk = torch.empty((TM1, field.vec_bytes(N)), dtype=torch.uint8, device=dev)
for rep in range(3):
    a, b = random.Random(rep), random.Random(rep)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    h = _native.mt_draw_coeffs(a, N, TM1)
    hd = torch.from_numpy(h).to(dev)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    ok = _native.mt_draw_coeffs_device(b, N, TM1, blk)
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    out[f"rep{rep}"] = {"host_draw_plus_h2d_s": t1 - t0, "device_draw_s": t2 - t1, "device_ok": ok,
                        "equal": bool(torch.equal(hd, blk)), "same_state": a.getstate() == b.getstate()}
    del h, hd
# fused draw + split (make_shares_vec's default path) vs draw then split, 3-of-5
sec = torch.randint(-(1 << 62), 1 << 62, (N,), dtype=torch.int64, device=dev)
sh = torch.empty((5, field.vec_bytes(N)), dtype=torch.uint8, device=dev)
for rep in range(3):
    a, b = random.Random(100 + rep), random.Random(100 + rep)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ok = _native.mt_split_device(a, sec, sh, N, 3, 5)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    ok2 = _native.mt_draw_coeffs_device(b, N, TM1, blk)
    _native.split_u64(sec, blk, sh, N, 3, 5)
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    out[f"split_rep{rep}"] = {"fused_draw_split_s": t1 - t0, "draw_then_split_s": t2 - t1, "ok": ok and ok2,
                              "same_state": a.getstate() == b.getstate()}
print(json.dumps(out))
