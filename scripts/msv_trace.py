#!/usr/bin/env python3
"""A short make_shares_vec(2^24, 5) loop for a HIP API + kernel trace
(rocprofv3 --hip-runtime-trace --kernel-trace --memory-copy-trace): where
the time between one call's generation and the next one's goes.  Marks the
timed calls with time.perf_counter_ns() stamps (one JSON line)."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "delta-node_amd"))

import torch  # noqa: E402

from delta_node.crypto import shamir  # noqa: E402

dev = torch.device("cuda", 0)
torch.cuda.set_device(0)
N = 1 << int(os.environ.get("LOG2N", "24"))
sec = torch.randint(-(1 << 62), 1 << 62, (N,), dtype=torch.int64, device=dev)
ss = shamir.SecretShare(3)
ss.random.seed(7)
for _ in range(4):
    r = ss.make_shares_vec(sec, 5)
    del r
torch.cuda.synchronize()
stamps = []
for _ in range(int(os.environ.get("REPS", "12"))):
    t0 = time.perf_counter_ns()
    r = ss.make_shares_vec(sec, 5)
    t1 = time.perf_counter_ns()
    del r
    stamps.append((t0, t1))
torch.cuda.synchronize()
print(json.dumps({"calls_us": [(b - a) / 1e3 for a, b in stamps]}))
