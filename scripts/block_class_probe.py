#!/usr/bin/env python3
"""Which share blocks land in the slow placement class, and does anything we
choose predict it?  Under the tuning library (DN_SHAMIR_LIB), allocates
PER 2 MiB-chunk blocks (memory.chunked_block, unpooled) at each virtual-range
alignment in ALIGNS (DN_BLOCK_ALIGN_LOG2) plus PER torch.empty blocks, and
per block records its address, the write-only stream rate over its 5 share
rows (dn_diag_tile_stream with no inputs, fastest grid) and the 3-of-5 split
of 2^24 into it (best of 4).  One JSON line per block, then a summary."""
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

assert "tuning" in _native.lib_path(), "run with DN_SHAMIR_LIB=.../libdn_shamir_tuning.so"
PER = int(os.environ.get("PER", "6"))
ALIGNS = [int(a) for a in os.environ.get("ALIGNS", "21,30").split(",")]
N = 1 << 24
dev = torch.device("cuda", 0)
torch.cuda.set_device(0)
stream = torch.cuda.current_stream()
vb = field.vec_bytes(N)
sec = torch.randint(-(1 << 62), 1 << 62, (N,), dtype=torch.int64, device=dev)
ss = shamir.SecretShare(3)
ss.random.seed(1)
co = ss.draw_coeffs_vec(N, dev)
blocks = []
for al in ALIGNS:
    os.environ["DN_BLOCK_ALIGN_LOG2"] = str(al)
    for _ in range(PER):
        blocks.append((f"chunk2M_align{al}", memory.chunked_block((5, vb), device=dev, pooled=False)))
os.environ.pop("DN_BLOCK_ALIGN_LOG2", None)
for _ in range(max(2, PER // 2)):
    blocks.append(("torch.empty", torch.empty((5, vb), dtype=torch.uint8, device=dev)))


def t_split(sh):
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


rows = []
for i, (kind, b) in enumerate(blocks):
    w = stream_ceiling([], [], [b[x] for x in range(5)], [66 * 256] * 5, N // 256, reps=3)
    sp = t_split(b)
    r = {"i": i, "kind": kind, "ptr": hex(b.data_ptr()), "ptr_mod_1G": b.data_ptr() % (1 << 30),
         "write_TBps": 5 * vb / (w["ms"] * 1e-3) / 1e12, "split_ms": sp, "split_frac": N * 470 / (sp * 1e-3) / 8e12}
    rows.append(r)
    print(json.dumps(r), flush=True)
summ = {}
for kind in sorted({r["kind"] for r in rows}):
    fr = sorted(r["split_frac"] for r in rows if r["kind"] == kind)
    summ[kind] = {"n": len(fr), "min": fr[0], "median": fr[len(fr) // 2], "max": fr[-1],
                  "n_ge_0_75": sum(f >= 0.75 for f in fr)}
print(json.dumps({"summary": summ}))
