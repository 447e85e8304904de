#!/usr/bin/env python3
"""make_shares_vec loops with the Python package at PKG (argv[1], the
directory holding delta_node/) over the product library: ms per call at 2^20
and 2^24, default pooled out and one caller block, after 4 warm-up calls.
For alternating-process A/Bs of host-side changes.  One JSON line."""
import json
import os
import sys
import time

PKG = os.path.abspath(sys.argv[1])
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("DN_SHAMIR_LIB", os.path.join(ROOT, "delta-node_amd", "lib", "libdn_shamir.so"))
sys.path.insert(0, PKG)

import torch  # noqa: E402

from delta_node.crypto import shamir  # noqa: E402
from delta_node.crypto.shamir import field  # noqa: E402

dev = torch.device("cuda", 0)
torch.cuda.set_device(0)
res = {"pkg": sys.argv[1]}
for lg, reps in ((20, 100), (24, 20)):
    n = 1 << lg
    sec = torch.randint(-(1 << 62), 1 << 62, (n,), dtype=torch.int64, device=dev)
    ss = shamir.SecretShare(3)
    ss.random.seed(lg)
    for _ in range(4):
        r = ss.make_shares_vec(sec, 5)
        del r
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        r = ss.make_shares_vec(sec, 5)
        del r
    torch.cuda.synchronize()
    res[f"2^{lg}_default_out_ms"] = (time.perf_counter() - t0) / reps * 1e3
    out = torch.empty((5, field.vec_bytes(n)), dtype=torch.uint8, device=dev)
    for _ in range(4):
        ss.make_shares_vec(sec, 5, out=out)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        ss.make_shares_vec(sec, 5, out=out)
    torch.cuda.synchronize()
    res[f"2^{lg}_caller_out_ms"] = (time.perf_counter() - t0) / reps * 1e3
    del out
print(json.dumps(res), flush=True)
