#!/usr/bin/env python3
"""make_shares_vec back to back, as a caller splitting vector after vector
with one SecretShare does (the case DN_MT_SPEC speculates on), under one
library (DN_SHAMIR_LIB): wall ms per call over 20 calls after 3 warm-up
calls, no device synchronisation inside the loop, at 2^12 .. 2^24 (3-of-5,
one caller torch.empty block per size, and from 2^22 also the default
out=None); and single calls on fresh
SecretShare objects (nothing to speculate on: the cost of a lone call).
Checks the loop's last output and state against draw-then-split.  One JSON
line."""
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
res = {"lib": os.path.basename(_native.lib_path())}
sec = torch.randint(-(1 << 62), 1 << 62, (1 << 24,), dtype=torch.int64, device=dev)
ok = True
for lg in [int(x) for x in os.environ.get("SIZES", "12,16,20,22,23,24").split(",")]:
    n = 1 << lg
    x = sec[:n]
    out = torch.empty((5, field.vec_bytes(n)), dtype=torch.uint8, device=dev)
    ss = shamir.SecretShare(3)
    ss.random.seed(lg)
    for _ in range(3):
        ss.make_shares_vec(x, 5, out=out)
    torch.cuda.synchronize()
    reps = 20
    t0 = time.perf_counter()
    for _ in range(reps):
        ss.make_shares_vec(x, 5, out=out)
    torch.cuda.synchronize()
    res[f"2^{lg}_loop_ms"] = (time.perf_counter() - t0) / reps * 1e3
    if lg >= 22:  # the product default out=None: each call's block from memory.share_block
        for _ in range(3):
            r = ss.make_shares_vec(x, 5)
            del r
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            r = ss.make_shares_vec(x, 5)
            del r
        torch.cuda.synchronize()
        res[f"2^{lg}_loop_default_out_ms"] = (time.perf_counter() - t0) / reps * 1e3
    # the loop's last call against draw then split from the state before it
    ref = shamir.SecretShare(3)
    ref.random.setstate(ss.random.getstate())
    got = ss.make_shares_vec(x, 5, out=out)
    co = ref.draw_coeffs_vec(n, dev)
    want = torch.empty_like(out)
    _native.split_u64(x, co, want, n, 3, 5)
    ok = ok and bool(torch.equal(got, want)) and ss.random.getstate() == ref.random.getstate()
    # lone calls: fresh objects (a speculation never applies)
    ts = []
    for r in range(6):
        f = shamir.SecretShare(3)
        f.random.seed(1000 + r)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        f.make_shares_vec(x, 5, out=out)
        torch.cuda.synchronize()
        if r:
            ts.append((time.perf_counter() - t0) * 1e3)
    res[f"2^{lg}_lone_ms"] = min(ts)
    if lg >= 20:  # lone calls into a pooled share block (the placement make_shares_vec allocates)
        pb = memory.share_block((5, field.vec_bytes(n)), dev)
        ts = []
        for r in range(6):
            f = shamir.SecretShare(3)
            f.random.seed(2000 + r)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            f.make_shares_vec(x, 5, out=pb)
            torch.cuda.synchronize()
            if r:
                ts.append((time.perf_counter() - t0) * 1e3)
        res[f"2^{lg}_lone_pooled_ms"] = min(ts)
        del pb
    del out, want, co
res["equal_draw_then_split"] = ok
try:
    res["spec_stats"] = _native.mt_spec_stats()
except Exception as e:  # an older library without the counters
    res["spec_stats"] = str(e)[:80]
print(json.dumps(res))
