#!/usr/bin/env python3
"""Does running the reconstruct of one batch beside the split of the next
(two streams, two share blocks) beat running them back to back?  Times K
steps each way on the same buffers (diagnostic for DESIGN.md §5)."""
import json
import os
import sys
import time

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
blocks = [torch.empty((5, field.vec_bytes(N)), dtype=torch.uint8, device=dev) for _ in range(2)]
recs = [torch.empty(N, dtype=torch.int64, device=dev) for _ in range(2)]
w = _native.lagrange([1, 3, 5], 3)
K = 20
sa, sb = torch.cuda.Stream(), torch.cuda.Stream()


def seq():
    for i in range(K):
        b = blocks[i % 2]
        _native.split_u64(sec, coeffs, b, N, 3, 5)
        _native.reconstruct([b[0], b[2], b[4]], w, out_u64=recs[i % 2], n=N)


def piped():
    # split i on stream A; reconstruct i on stream B after split i, beside split i+1
    ev_split = [torch.cuda.Event() for _ in range(K)]
    ev_rec = [torch.cuda.Event() for _ in range(K)]
    for i in range(K):
        b = blocks[i % 2]
        with torch.cuda.stream(sa):
            if i >= 2:
                sa.wait_event(ev_rec[i - 2])  # block i%2 free again
            _native.split_u64(sec, coeffs, b, N, 3, 5)
            ev_split[i].record(sa)
        with torch.cuda.stream(sb):
            sb.wait_event(ev_split[i])
            _native.reconstruct([b[0], b[2], b[4]], w, out_u64=recs[i % 2], n=N)
            ev_rec[i].record(sb)


res = {}
for name, fn in (("sequential", seq), ("pipelined", piped), ("sequential2", seq), ("pipelined2", piped)):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    fn()
    torch.cuda.synchronize()
    res[name + "_ms_per_step"] = (time.perf_counter() - t0) / K * 1e3
res["roundtrip"] = bool(torch.equal(recs[0], sec) and torch.equal(recs[1], sec))
print(json.dumps(res))
