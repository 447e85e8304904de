#!/usr/bin/env python3
"""The headline step on one GPU's shard of the 2^24 vector at N = 2/4/8
(2^23 / 2^22 / 2^21 elements): under the tuning library
(DN_SHAMIR_LIB), per size the split's grid cap (DN_GRID_CAP) and wave
schedule (DN_TILE_MAP) and the reconstruct's grid cap, each timed by HIP
events as the median of REPS launches over 3 share blocks, plus the bench's
own step (split + reconstruct back to back, 20 steps) per split setting.
One JSON line per (size, setting)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "delta-node_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from delta_node.crypto import shamir  # noqa: E402
from delta_node.crypto.shamir import _native, field, memory  # noqa: E402

assert "tuning" in _native.lib_path(), "run with DN_SHAMIR_LIB=.../libdn_shamir_tuning.so"
REPS = int(os.environ.get("REPS", "10"))
SIZES = [int(x) for x in os.environ.get("SIZES", "21,22,23").split(",")]
CAPS = [int(x) for x in os.environ.get("CAPS", "0,512,1024,2048,4096").split(",")]
MAPS = [int(x) for x in os.environ.get("MAPS", "0,1").split(",")]
dev = torch.device("cuda", 0)
torch.cuda.set_device(0)
stream = torch.cuda.current_stream()
w = _native.lagrange([1, 3, 5], 3)


def timed(fn, reps):
    ts = []
    for _ in range(reps):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record(stream)
        fn()
        e.record(stream)
        e.synchronize()
        ts.append(s.elapsed_time(e))
    return float(np.median(ts))


def setenv(k, v):
    if v is None:
        os.environ.pop(k, None)
    else:
        os.environ[k] = str(v)


for lg in SIZES:
    N = 1 << lg
    vb = field.vec_bytes(N)
    sec = torch.randint(-(1 << 62), 1 << 62, (N,), dtype=torch.int64, device=dev)
    ss = shamir.SecretShare(3)
    ss.random.seed(lg)
    co = ss.draw_coeffs_vec(N, dev)
    blocks = [memory.share_block((5, vb), dev) for _ in range(3)]
    rec = torch.empty(N, dtype=torch.int64, device=dev)
    rows = [[b[0], b[2], b[4]] for b in blocks]
    for b in blocks:
        _native.split_u64(sec, co, b, N, 3, 5)
    torch.cuda.synchronize()
    for cap in CAPS:
        for mp in MAPS:
            setenv("DN_GRID_CAP", cap or None)
            setenv("DN_TILE_MAP", mp)
            sp = [timed(lambda b=b: _native.split_u64(sec, co, b, N, 3, 5), REPS) for b in blocks]
            rc = [timed(lambda r=r: _native.reconstruct(r, w, out_u64=rec, n=N), REPS) for r in rows]
            # the bench's step: split + reconstruct back to back, 20 steps rotating over the blocks
            for i in range(3):
                _native.split_u64(sec, co, blocks[i % 3], N, 3, 5)
                _native.reconstruct(rows[i % 3], w, out_u64=rec, n=N)
            torch.cuda.synchronize()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record(stream)
            for i in range(20):
                _native.split_u64(sec, co, blocks[i % 3], N, 3, 5)
                _native.reconstruct(rows[i % 3], w, out_u64=rec, n=N)
            e.record(stream)
            e.synchronize()
            step = s.elapsed_time(e) / 20
            ok = bool(torch.equal(rec, sec))
            print(json.dumps({"log2n": lg, "cap": cap, "map": mp, "split_ms": sp, "recon_ms": rc,
                              "step_ms": step, "elems_per_s": N / (step * 1e-3), "roundtrip": ok}), flush=True)
    setenv("DN_GRID_CAP", None)
    setenv("DN_TILE_MAP", None)
    del blocks, rows, co, sec, rec
    torch.cuda.empty_cache()
