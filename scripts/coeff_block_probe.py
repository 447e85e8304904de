#!/usr/bin/env python3
"""Does the coefficient block's placement move the headline split?  3-of-5
split of 2^24 (dn_m521_split_u64, 470 B/element) into three share blocks
(memory.share_block), the same coefficients read from a torch.empty block or
from a 2 MiB-chunk block (memory.share_block), alternating, HIP events, best
of 5 per (share block, coefficient block), two rounds.  One JSON line each."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "delta-node_amd"))

import torch  # noqa: E402

from delta_node.crypto import shamir  # noqa: E402
from delta_node.crypto.shamir import _native, field, memory  # noqa: E402

N = 1 << 24
dev = torch.device("cuda", 0)
torch.cuda.set_device(0)
stream = torch.cuda.current_stream()
vb = field.vec_bytes(N)
sec = torch.randint(-(1 << 62), 1 << 62, (N,), dtype=torch.int64, device=dev)
ss = shamir.SecretShare(3)
ss.random.seed(1)
co_e = ss.draw_coeffs_vec(N, dev)
co_c = memory.share_block(tuple(co_e.shape), dev)
co_c.copy_(co_e)
shares = [memory.share_block((5, vb), dev) for _ in range(3)]


def t_split(co, sh):
    _native.split_u64(sec, co, sh, N, 3, 5)
    best = None
    for _ in range(5):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record(stream)
        _native.split_u64(sec, co, sh, N, 3, 5)
        e.record(stream)
        torch.cuda.synchronize()
        best = s.elapsed_time(e) if best is None else min(best, s.elapsed_time(e))
    return best


for rnd in range(2):
    for i, sh in enumerate(shares):
        r = {"round": rnd, "share_block": i, "coeffs_torch_empty_ms": t_split(co_e, sh),
             "coeffs_share_block_ms": t_split(co_c, sh)}
        r["frac_empty"] = N * 470 / (r["coeffs_torch_empty_ms"] * 1e-3) / 8e12
        r["frac_chunked"] = N * 470 / (r["coeffs_share_block_ms"] * 1e-3) / 8e12
        print(json.dumps(r), flush=True)
print(json.dumps({"equal": bool(torch.equal(co_c, co_e))}))
