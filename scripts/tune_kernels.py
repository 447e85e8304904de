#!/usr/bin/env python3
"""Interleaved A/B sweep of launch geometry (DN_GRID_CAP) for split/reconstruct,
in one process (cdna guide rule 24).  Prints one JSON line per config."""
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

N = 1 << int(os.environ.get("LOG2N", "24"))
caps = [int(c) for c in os.environ.get("CAPS", "1024,2048,4096,8192,16384").split(",")]
rounds = int(os.environ.get("ROUNDS", "5"))
dev = torch.device("cuda", 0)
rng = np.random.default_rng(1)
sec = torch.from_numpy(rng.integers(-(1 << 63), (1 << 63) - 1, size=N, endpoint=True, dtype=np.int64)).to(dev)
ss = shamir.SecretShare(3)
ss.random.seed(1)
coeffs = ss.draw_coeffs_vec(N, dev)
shares = torch.empty((5, field.vec_bytes(N)), dtype=torch.uint8, device=dev)
rec = torch.empty(N, dtype=torch.int64, device=dev)
configs = {"135": ([1, 3, 5], [0, 2, 4]), "245": ([2, 4, 5], [1, 3, 4]), "123": ([1, 2, 3], [0, 1, 2])}
res = {}


def timeit(fn, iters=10):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


unrolls = os.environ.get("UNROLLS", "1,0").split(",")
for r in range(rounds):
    for cap, unroll in [(c, u) for c in caps for u in unrolls]:
        os.environ["DN_GRID_CAP"] = str(cap)
        os.environ["DN_RECON_UNROLL"] = unroll
        for horner in ("0", "1"):
            os.environ["DN_SPLIT_HORNER"] = horner
            t_split = timeit(lambda: _native.split_u64(sec, coeffs, shares, N, 3, 5))
            res.setdefault((cap, "split_horner" if horner == "1" else "split_fd", unroll), []).append(t_split)
        os.environ["DN_SPLIT_HORNER"] = "0"
        for name, (xs, rows) in configs.items():
            w = _native.lagrange(xs, 3)
            t_rec = timeit(lambda: _native.reconstruct([shares[i] for i in rows], w, out_u64=rec, n=N))
            res.setdefault((cap, "rec" + name, unroll), []).append(t_rec)
for (cap, kind, unroll), ts in sorted(res.items()):
    b = N * (470 if kind.startswith("split") else 206)
    print(json.dumps({"cap": cap, "kernel": kind, "recon_unroll": unroll, "ms_median": float(np.median(ts)),
                      "ms_min": float(np.min(ts)),
                      "GBps_median": b / (np.median(ts) * 1e-3) / 1e9}))
