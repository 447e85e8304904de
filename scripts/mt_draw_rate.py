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
print(json.dumps(out))
