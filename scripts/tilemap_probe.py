#!/usr/bin/env python3
"""Split / reconstruct duration per share allocation under each wave schedule
(DN_TILE_MAP=0 cyclic, 1 XCD-contiguous, 2 blocked, 3 workgroup-cooperative;
MODES=0,1,2,3) and optional grid caps (CAPS=0,16384; 0 = library default),
interleaved in one process so every mode sees the same allocations."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "delta-node_amd"))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from delta_node.crypto import shamir  # noqa: E402
from delta_node.crypto.shamir import _native, field  # noqa: E402

N = 1 << 24
dev = torch.device("cuda", 0)
rng = np.random.default_rng(1)
sec = torch.from_numpy(rng.integers(-(1 << 63), (1 << 63) - 1, size=N, endpoint=True, dtype=np.int64)).to(dev)
ss = shamir.SecretShare(3)
ss.random.seed(1)
coeffs = ss.draw_coeffs_vec(N, dev)
rec = torch.empty(N, dtype=torch.int64, device=dev)
w135 = _native.lagrange([1, 3, 5], 3)
sets = [torch.empty((5, field.vec_bytes(N)), dtype=torch.uint8, device=dev) for _ in range(int(os.environ.get("SETS", "6")))]
stream = torch.cuda.current_stream()
MODES = [f"{m}/{c}" for m in os.environ.get("MODES", "0,1,2,3").split(",") for c in os.environ.get("CAPS", "0").split(",")]


def timed(fn, iters=8):
    fn()
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(iters)]
    for a, b in evs:
        a.record(stream)
        fn()
        b.record(stream)
    torch.cuda.synchronize()
    return [a.elapsed_time(b) for a, b in evs]


res = {}
for rnd in range(3):
    for i, sh in enumerate(sets):
        for m in MODES:
            os.environ["DN_TILE_MAP"] = m.split("/")[0]
            cap = m.split("/")[1] if "/" in m else "0"
            os.environ["DN_GRID_CAP"] = cap
            res.setdefault((i, m, "split"), []).extend(timed(lambda: _native.split_u64(sec, coeffs, sh, N, 3, 5)))
            rows = [sh[0], sh[2], sh[4]]
            res.setdefault((i, m, "recon"), []).extend(timed(lambda: _native.reconstruct(rows, w135, out_u64=rec, n=N)))
            assert torch.equal(rec, sec)
for (i, m, k), ts in sorted(res.items()):
    print(json.dumps({"set": i, "tile_map": m, "kernel": k, "ms_median": float(np.median(ts)),
                      "min": float(np.min(ts)), "max": float(np.max(ts))}), flush=True)
