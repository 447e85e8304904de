#!/usr/bin/env python3
"""Does the share block's placement need 2 MiB physical chunks, or do larger
chunks (fewer hipMemCreate / hipMemMap calls: the cold first call maps ~2,640
per 5.5 GB block) run as fast?  Per chunk size in CHUNKS (MiB), PER unpooled,
unprobed blocks of 5 x vec_bytes(2^24) (all kept alive, so no block reuses
another's pages): the allocation's wall time, the allocator's row-order write
probe (memory._write_rate) and the 3-of-5 split into it (best of 3).  One
JSON line per block, then a summary per chunk size."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "delta-node_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from delta_node.crypto import shamir  # noqa: E402
from delta_node.crypto.shamir import _native, field, memory  # noqa: E402

PER = int(os.environ.get("PER", "6"))
CHUNKS = [int(c) for c in os.environ.get("CHUNKS", "2,4,8,16").split(",")]
N = 1 << 24
dev = torch.device("cuda", 0)
torch.cuda.set_device(0)
vb = field.vec_bytes(N)
sec = torch.randint(-(1 << 62), 1 << 62, (N,), dtype=torch.int64, device=dev)
ss = shamir.SecretShare(3)
ss.random.seed(1)
co = ss.draw_coeffs_vec(N, dev)
BYTES = N * 470
stream = torch.cuda.current_stream()
keep = []
rows = []
for rnd in range(PER):
    for mib in CHUNKS:  # interleaved: each size draws from the same stretch of the pool
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        blk = memory.chunked_block((5, vb), mib << 20, dev, pooled=False)
        torch.cuda.synchronize()
        alloc_ms = (time.perf_counter() - t0) * 1e3
        rate = memory._write_rate(blk.data_ptr(), blk.numel(), dev, (5, vb))
        best = None
        for _ in range(4):
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record(stream)
            _native.split_u64(sec, co, blk, N, 3, 5)
            e.record(stream)
            e.synchronize()
            ms = s.elapsed_time(e)
            best = ms if best is None else min(best, ms)
        r = {"round": rnd, "chunk_MiB": mib, "alloc_ms": alloc_ms, "probe_TBps": rate / 1e12, "split_ms": best,
             "split_frac": BYTES / (best * 1e-3) / 8e12}
        rows.append(r)
        print(json.dumps(r), flush=True)
        keep.append(blk)
summ = {}
for mib in CHUNKS:
    fr = [r["split_frac"] for r in rows if r["chunk_MiB"] == mib]
    al = [r["alloc_ms"] for r in rows if r["chunk_MiB"] == mib]
    summ[mib] = {"frac_min": min(fr), "frac_median": float(np.median(fr)), "frac_max": max(fr),
                 "n_ge_0_78": sum(f >= 0.78 for f in fr), "alloc_ms_median": float(np.median(al))}
print(json.dumps({"summary": summ}), flush=True)
