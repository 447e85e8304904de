#!/usr/bin/env python3
"""Split duration per share allocation vs launch size (DN_GRID_CAP caps the
workgroups; below 2048 it also caps the resident waves)."""
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
sets = [torch.empty((5, field.vec_bytes(N)), dtype=torch.uint8, device=dev) for _ in range(int(os.environ.get("SETS", "6")))]
stream = torch.cuda.current_stream()
CAPS = os.environ.get("CAPS", "256,512,768,1024,1536,2048,16384").split(",")


def timed(fn, iters=6):
    fn()
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(iters)]
    for a, b in evs:
        a.record(stream)
        fn()
        b.record(stream)
    torch.cuda.synchronize()
    return [a.elapsed_time(b) for a, b in evs]


res = {}
for rnd in range(2):
    for i, sh in enumerate(sets):
        for cap in CAPS:
            for tm in os.environ.get("TILE_MAPS", "0").split(","):
                os.environ["DN_GRID_CAP"] = cap
                os.environ["DN_TILE_MAP"] = tm
                res.setdefault((i, int(cap), tm), []).extend(
                    timed(lambda: _native.split_u64(sec, coeffs, sh, N, 3, 5)))
for (i, cap, tm), ts in sorted(res.items()):
    print(json.dumps({"set": i, "cap": cap, "tile_map": tm, "ms_median": float(np.median(ts)),
                      "min": float(np.min(ts))}), flush=True)
