#!/usr/bin/env python3
"""make_shares_vec (3-of-5, shares preallocated) called 8 times per size, with
a 3 ms host sleep between calls, for a kernel + memory-copy trace of one
call's GPU timeline (rocprofv3 --kernel-trace --memory-copy-trace): the jump
levels, the generation, the small copies and the gaps between them
(scripts/msv_trace_summary.py).  Prints the wall time per call.
usage: msv_trace.py [log2n ...]   (default 24)"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "delta-node_amd"))

import torch  # noqa: E402

from delta_node.crypto import shamir  # noqa: E402
from delta_node.crypto.shamir import field  # noqa: E402

dev = torch.device("cuda", 0)
res = {}
for lg in [int(a) for a in sys.argv[1:]] or [24]:
    N = 1 << lg
    sec = torch.randint(-(1 << 62), 1 << 62, (N,), dtype=torch.int64, device=dev)
    sh = torch.empty((5, field.vec_bytes(N)), dtype=torch.uint8, device=dev)
    ss = shamir.SecretShare(3)
    ss.random.seed(24)
    walls = []
    for _ in range(8):
        torch.cuda.synchronize()
        time.sleep(0.003)
        t0 = time.perf_counter()
        ss.make_shares_vec(sec, 5, out=sh)
        torch.cuda.synchronize()
        walls.append((time.perf_counter() - t0) * 1e3)
    res[f"2^{lg}"] = walls
    time.sleep(0.01)
print(json.dumps({"make_shares_vec_wall_ms": res}))
