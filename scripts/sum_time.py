#!/usr/bin/env python3
"""The coordinator's member sum alone (dn_i64_sum, 10 int64 members of 2^24),
HIP events, best of 3 rounds of 10 calls, under the library DN_SHAMIR_LIB
selects (A/B).  One JSON line."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "delta-node_amd"))

import torch  # noqa: E402

from delta_node.crypto.shamir import _native  # noqa: E402
from delta_node.utils import sum_int64  # noqa: E402

n, k = 1 << 24, int(os.environ.get("MEMBERS", "10"))
dev = torch.device("cuda", 0)
mem = [torch.randint(-2**62, 2**62, (n,), dtype=torch.int64, device=dev) for _ in range(k)]
out = torch.empty(n, dtype=torch.int64, device=dev)
for _ in range(3):
    sum_int64(mem, out=out)
best = None
for _ in range(3):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(10):
        sum_int64(mem, out=out)
    e.record()
    e.synchronize()
    ms = s.elapsed_time(e) / 10
    best = ms if best is None else min(best, ms)
ok = bool(torch.equal(out, torch.stack(mem).sum(0)))
print(json.dumps({"lib": os.path.basename(_native.lib_path()), "members": k, "ms": best,
                  "frac_of_8TBps": (k + 1) * 8 * n / (best * 1e-3) / 8e12, "equal": ok}))
