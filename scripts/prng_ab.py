#!/usr/bin/env python3
"""Device-PRNG split (dn_m521_split_prng, 3-of-5, 2^24 int64) kernel time of
one library (DN_SHAMIR_LIB selects it) for ChaCha20 / 12 / 8, HIP events on
the launch stream, best of 3 rounds of 5 launches, round trip checked.
Prints one JSON line."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "delta-node_amd"))

import torch  # noqa: E402

from delta_node.crypto import shamir  # noqa: E402
from delta_node.crypto.shamir import _native, field  # noqa: E402

n = 1 << 24
dev = torch.device("cuda", 0)
g = torch.Generator(device=dev)
g.manual_seed(3)
sec = torch.randint(-(1 << 62), 1 << 62, (n,), dtype=torch.int64, device=dev, generator=g)
sh = torch.empty((5, field.vec_bytes(n)), dtype=torch.uint8, device=dev)
res = {"lib": os.path.basename(os.environ.get("DN_SHAMIR_LIB", "libdn_shamir.so"))}
ss = shamir.SecretShare(3)
for rounds in (20, 12, 8):
    best = None
    for _ in range(3):
        _native.split_prng(sec, bytes(range(32)), 0, rounds, 0, sh, n, 3, 5)
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(5):
            _native.split_prng(sec, bytes(range(32)), 0, rounds, 0, sh, n, 3, 5)
        e.record()
        torch.cuda.synchronize()
        ms = s.elapsed_time(e) / 5
        best = ms if best is None else min(best, ms)
    back = ss.resolve_shares_vec([sh[1], sh[2], sh[4]], [2, 3, 5], n)
    res[f"chacha{rounds}_ms"] = best
    res[f"chacha{rounds}_hbm_frac"] = n * 338 / (best * 1e-3) / 8e12
    res[f"chacha{rounds}_roundtrip"] = bool(torch.equal(back, sec))
print(json.dumps(res))
