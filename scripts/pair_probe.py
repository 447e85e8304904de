#!/usr/bin/env python3
"""Is a share block's slowness its own, or its pair's with the coefficient
block?  Maps PER 2 MiB-chunk share blocks (unprobed) and two coefficient
blocks (2 MiB-chunk and torch.empty); per share block: the split time with
each coefficient block, the write-only fill rate, and a read+write stream
rate (dn_diag_tile_stream: a fixed torch.empty source's 1/3 read per 2/3
written, the split's mix) — which of them predicts the split?"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "delta-node_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from bench import stream_ceiling  # noqa: E402
from delta_node.crypto import shamir  # noqa: E402
from delta_node.crypto.shamir import _native, field, memory  # noqa: E402

PER = int(os.environ.get("PER", "8"))
N = 1 << 24
dev = torch.device("cuda", 0)
torch.cuda.set_device(0)
stream = torch.cuda.current_stream()
vb = field.vec_bytes(N)
sec = torch.randint(-(1 << 62), 1 << 62, (N,), dtype=torch.int64, device=dev)
ss = shamir.SecretShare(3)
ss.random.seed(1)
co_c = memory.chunked_block((2, vb), device=dev, pooled=False)
co_c.copy_(ss.draw_coeffs_vec(N, dev))
co_e = co_c.clone()  # torch.empty memory
src = torch.empty(2 * vb, dtype=torch.uint8, device=dev)  # fixed read source of the mixed probe
blocks = [memory.chunked_block((5, vb), device=dev, pooled=False) for _ in range(PER)]


def t_split(co, sh):
    _native.split_u64(sec, co, sh, N, 3, 5)
    best = None
    for _ in range(4):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record(stream)
        _native.split_u64(sec, co, sh, N, 3, 5)
        e.record(stream)
        torch.cuda.synchronize()
        best = s.elapsed_time(e) if best is None else min(best, s.elapsed_time(e))
    return best


for i, b in enumerate(blocks):
    w = stream_ceiling([], [], [b[x] for x in range(5)], [66 * 256] * 5, N // 256, reps=3)
    m = stream_ceiling([src[:vb], src[vb:]], [66 * 256] * 2, [b[x] for x in range(5)], [66 * 256] * 5, N // 256,
                       reps=3)
    r = {"i": i, "ptr": hex(b.data_ptr()), "fill_TBps": 5 * vb / (w["ms"] * 1e-3) / 1e12,
         "mixed_TBps": 7 * vb / (m["ms"] * 1e-3) / 1e12,
         "split_ms_coeff_chunked": t_split(co_c, b), "split_ms_coeff_empty": t_split(co_e, b)}
    print(json.dumps(r), flush=True)
