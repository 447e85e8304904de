#!/usr/bin/env python3
"""Placement experiment: the 3-of-5 split of 2^24
elements and the fused MT draw + split (make_shares_vec) into share blocks
from torch.empty against blocks from memory.chunked_block (physical chunks
of 2 MiB / 64 MiB, and one whole-block handle), all in ONE process, two
alternating rounds.  Prints one JSON line per buffer per round, then a
summary line.  usage: block_probe.py [per_kind=5]"""
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

per = int(sys.argv[1]) if len(sys.argv) > 1 else 5
dev = torch.device("cuda", 0)
N, t, n = 1 << 24, 3, 5
vb = field.vec_bytes(N)
FE = 66
split_bytes = N * (8 + (t - 1) * FE + n * FE)
sec = torch.randint(-(1 << 62), 1 << 62, (N,), dtype=torch.int64, device=dev)
ss = shamir.SecretShare(t)
ss.random.seed(5)
coeffs = ss.draw_coeffs_vec(N, dev)
whole = (n * vb + (2 << 20) - 1) // (2 << 20) * (2 << 20)
t0 = time.time()
bufs = []
for k in range(per):
    bufs.append(("torch", torch.empty((n, vb), dtype=torch.uint8, device=dev)))
for k in range(per):
    bufs.append(("chunk2M", memory.chunked_block((n, vb), 2 << 20)))
for k in range(per):
    bufs.append(("chunk64M", memory.chunked_block((n, vb), 64 << 20)))
for k in range(max(1, per // 2)):
    bufs.append(("whole", memory.chunked_block((n, vb), whole)))
alloc_s = time.time() - t0
print(json.dumps({"alloc_s": alloc_s, "buffers": len(bufs), "granularity": memory.granularity(0)}), flush=True)
stream = torch.cuda.current_stream()
ref = None
for kind, b in bufs:  # first touch + parity: every buffer holds the same split
    _native.split_u64(sec, coeffs, b, N, t, n)
    if ref is None:
        ref = b.clone()
    assert torch.equal(b, ref), kind
del ref
torch.cuda.synchronize()


def time_split(b, reps=6):
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    for a, e in evs:
        a.record(stream)
        _native.split_u64(sec, coeffs, b, N, t, n)
        e.record(stream)
    torch.cuda.synchronize()
    return float(np.median([a.elapsed_time(e) for a, e in evs]))


def time_msv(b, reps=4):
    s2 = shamir.SecretShare(t)
    s2.random.seed(9)
    out = []
    for _ in range(reps):
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        s2.make_shares_vec(sec, n, out=b)
        torch.cuda.synchronize()
        out.append((time.perf_counter() - t1) * 1e3)
    return float(np.median(out))


res = {}
for rnd in range(2):
    for i, (kind, b) in enumerate(bufs):
        ms = time_split(b)
        m2 = time_msv(b)
        frac = split_bytes / (ms * 1e-3) / 8e12
        res.setdefault(kind, []).append((ms, frac, m2))
        print(json.dumps({"round": rnd, "buf": i, "kind": kind, "split_ms": ms, "frac": frac, "msv_ms": m2}),
              flush=True)
summ = {}
for kind, v in res.items():
    fr = [x[1] for x in v]
    summ[kind] = {"split_ms_median": float(np.median([x[0] for x in v])), "frac_min": min(fr),
                  "frac_median": float(np.median(fr)), "frac_max": max(fr), "n_ge_0_70": sum(f >= 0.70 for f in fr),
                  "n": len(fr), "msv_ms_median": float(np.median([x[2] for x in v]))}
print(json.dumps({"summary": summ}), flush=True)
