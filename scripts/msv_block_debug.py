#!/usr/bin/env python3
"""Debug: make_shares_vec's fused MT draw + split into a fresh share block
vs into torch.empty vs draw-then-split (tests/test_gpu_memory.py::
test_make_shares_vec_default_output_is_share_block failed in pass r04g).
Per trial: which rows / elements differ from the draw-then-split result.
Prints one JSON line per trial."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "delta-node_amd"))

import torch  # noqa: E402

from delta_node.crypto import shamir  # noqa: E402
from delta_node.crypto.shamir import _native, field, memory  # noqa: E402

dev = torch.device("cuda", 0)
torch.cuda.set_device(0)
N = 1 << int(os.environ.get("LOG2N", "18"))
vb = field.vec_bytes(N)
print(json.dumps({"lib": _native.lib_path(), "N": N}), flush=True)


def diff(x, ref):
    out = {}
    for r in range(ref.shape[0]):
        d = (x[r] != ref[r]).nonzero().flatten()
        if d.numel():
            b = d.cpu()
            out[r] = {"bytes": int(b.numel()), "first": int(b[0]), "last": int(b[-1]),
                      "first_tile": int(b[0]) // field.TILE_BYTES, "last_tile": int(b[-1]) // field.TILE_BYTES}
    return out


KINDS = os.environ.get("KINDS", "share_block,torch.empty,share_block_sync,chunked_nopool").split(",")


def overlaps(t):
    """torch caching-allocator segments whose address range meets t's"""
    a0, a1 = t.data_ptr(), t.data_ptr() + t.numel() * t.element_size()
    hits = []
    for sgm in torch.cuda.memory_snapshot():
        s0, s1 = sgm["address"], sgm["address"] + sgm["total_size"]
        if s0 < a1 and a0 < s1:
            hits.append([hex(s0), sgm["total_size"]])
    return hits


for trial in range(int(os.environ.get("TRIALS", "4"))):
    kind = KINDS[trial % len(KINDS)]
    sec = torch.randint(-(1 << 62), 1 << 62, (N,), dtype=torch.int64, device=dev)
    a, b = shamir.SecretShare(3), shamir.SecretShare(3)
    a.random.seed(11 + trial)
    b.random.seed(11 + trial)
    if kind == "torch.empty":
        out = torch.empty((5, vb), dtype=torch.uint8, device=dev)
        a.make_shares_vec(sec, 5, out=out)
    elif kind == "chunked_nopool":
        out = memory.chunked_block((5, vb), device=dev, pooled=False)
        out.fill_(0xEE)
        a.make_shares_vec(sec, 5, out=out)
    else:
        out = a.make_shares_vec(sec, 5)
    if kind == "share_block_sync":
        torch.cuda.synchronize()
    co = b.draw_coeffs_vec(N, dev)
    ref = torch.empty((5, vb), dtype=torch.uint8, device=dev)
    _native.split_u64(sec, co, ref, N, 3, 5)
    d = diff(out, ref)
    torch.cuda.synchronize()
    d2 = diff(out, ref)  # again, after a full device sync
    print(json.dumps({"trial": trial, "kind": kind, "ptr": hex(out.data_ptr()), "torch_segments_overlapping": overlaps(out),
                      "state_equal": a.random.getstate() == b.random.getstate(),
                      "diff": d, "diff_after_sync": d2, "pool": memory.pool_stats()}), flush=True)
    del out
