#!/usr/bin/env python3
"""Where the host time of make_shares_vec(2^24, out=None) goes in a loop:
the pooled block's acquire/release alone (memory.share_block + del) timed
per call, then cProfile of 20 back-to-back calls (top entries by total
time).  Prints JSON, then the profile table."""
import cProfile
import io
import json
import os
import pstats
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "delta-node_amd"))

import torch  # noqa: E402

from delta_node.crypto import shamir  # noqa: E402
from delta_node.crypto.shamir import field, memory  # noqa: E402

dev = torch.device("cuda", 0)
torch.cuda.set_device(0)
N = 1 << int(os.environ.get("LOG2N", "24"))
vb = field.vec_bytes(N)
sec = torch.randint(-(1 << 62), 1 << 62, (N,), dtype=torch.int64, device=dev)
res = {}
for _ in range(3):
    b = memory.share_block((5, vb), dev)
    del b
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(50):
    b = memory.share_block((5, vb), dev)
    del b
res["share_block_acquire_release_us"] = (time.perf_counter() - t0) / 50 * 1e6
ss = shamir.SecretShare(3)
ss.random.seed(1)
for _ in range(3):
    r = ss.make_shares_vec(sec, 5)
    del r
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(20):
    r = ss.make_shares_vec(sec, 5)
    del r
torch.cuda.synchronize()
res["loop_default_out_ms"] = (time.perf_counter() - t0) / 20 * 1e3
out = torch.empty((5, vb), dtype=torch.uint8, device=dev)
t0 = time.perf_counter()
for _ in range(20):
    ss.make_shares_vec(sec, 5, out=out)
torch.cuda.synchronize()
res["loop_caller_out_ms"] = (time.perf_counter() - t0) / 20 * 1e3
res["pool"] = {k: v for k, v in memory.pool_stats().items() if isinstance(v, (int, float))}
print(json.dumps(res), flush=True)
pr = cProfile.Profile()
pr.enable()
for _ in range(20):
    r = ss.make_shares_vec(sec, 5)
    del r
torch.cuda.synchronize()
pr.disable()
s = io.StringIO()
pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(25)
print(s.getvalue())
