#!/usr/bin/env python3
"""The headline reconstruct alone (xs {1,3,5} -> int64 at 2^24, share rows in a
memory.share_block block), HIP events on its stream, best of 3 rounds of 10
launches, under the library DN_SHAMIR_LIB selects (tuning knobs such as
DN_TILE_MAP apply with the tuning library).  One JSON line."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "delta-node_amd"))

import torch  # noqa: E402

from delta_node.crypto import shamir  # noqa: E402
from delta_node.crypto.shamir import _native, field, memory  # noqa: E402

N = 1 << int(os.environ.get("LOG2N", "24"))
dev = torch.device("cuda", 0)
sec = torch.randint(-(1 << 62), 1 << 62, (N,), dtype=torch.int64, device=dev)
ss = shamir.SecretShare(3)
ss.random.seed(3)
sh = memory.share_block((5, field.vec_bytes(N)), dev)
ss.make_shares_vec(sec, 5, out=sh)
xs = [1, 3, 5]
rows = [sh[x - 1] for x in xs]
w = _native.lagrange(xs, 3)
rec = torch.empty(N, dtype=torch.int64, device=dev)
for _ in range(3):
    _native.reconstruct(rows, w, out_u64=rec, n=N)
torch.cuda.synchronize()
best = None
for _ in range(3):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(10):
        _native.reconstruct(rows, w, out_u64=rec, n=N)
    e.record()
    e.synchronize()
    ms = s.elapsed_time(e) / 10
    best = ms if best is None else min(best, ms)
ok = bool(torch.equal(rec, sec))
print(json.dumps({"lib": os.path.basename(_native.lib_path()), "tile_map": os.environ.get("DN_TILE_MAP"),
                  "ms": best, "frac_of_8TBps": N * (3 * 66 + 8) / (best * 1e-3) / 8e12, "equal": ok}))
