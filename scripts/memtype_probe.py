#!/usr/bin/env python3
"""Split / reconstruct duration vs the share buffer's memory type: torch
(default coarse-grained), hipExtMallocWithFlags(hipDeviceMallocUncached) and
(hipDeviceMallocFinegrained); several allocations each, interleaved."""
import ctypes
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
VB = field.vec_bytes(N)
dev = torch.device("cuda", 0)
rng = np.random.default_rng(1)
sec = torch.from_numpy(rng.integers(-(1 << 63), (1 << 63) - 1, size=N, endpoint=True, dtype=np.int64)).to(dev)
ss = shamir.SecretShare(3)
ss.random.seed(1)
coeffs = ss.draw_coeffs_vec(N, dev)
rec = torch.empty(N, dtype=torch.int64, device=dev)
w135 = _native.lagrange([1, 3, 5], 3)
hip = ctypes.CDLL("libamdhip64.so")
stream = torch.cuda.current_stream()


class Raw:
    def __init__(self, p):
        self.p = p

    def data_ptr(self):
        return self.p


def hip_alloc(nbytes, flags):
    p = ctypes.c_void_p()
    rc = hip.hipExtMallocWithFlags(ctypes.byref(p), ctypes.c_size_t(nbytes), flags)
    if rc != 0:
        raise RuntimeError(f"hipExtMallocWithFlags({flags}) rc={rc}")
    return p.value


sets = []
for kind, count in (("torch", 3), ("uncached", 3), ("finegrained", 1)):
    for _ in range(count):
        if kind == "torch":
            sets.append((kind, torch.empty(5 * VB, dtype=torch.uint8, device=dev)))
        else:
            try:
                sets.append((kind, Raw(hip_alloc(5 * VB, 3 if kind == "uncached" else 1))))
            except RuntimeError as e:
                print(json.dumps({"kind": kind, "error": str(e)}), flush=True)


def timed(fn, iters=8):
    fn()
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(iters)]
    for a, b in evs:
        a.record(stream)
        fn()
        b.record(stream)
    torch.cuda.synchronize()
    return [a.elapsed_time(b) for a, b in evs]


res = {}
for rnd in range(3):
    for i, (kind, buf) in enumerate(sets):
        base = buf.data_ptr()
        rows = [Raw(base + r * VB) for r in (0, 2, 4)]
        res.setdefault((i, kind, "split"), []).extend(
            timed(lambda: _native.split_u64(sec, coeffs, Raw(base), N, 3, 5)))
        res.setdefault((i, kind, "recon"), []).extend(
            timed(lambda: _native.reconstruct(rows, w135, out_u64=rec, n=N)))
        assert torch.equal(rec, sec)
for (i, kind, k), ts in sorted(res.items()):
    print(json.dumps({"set": i, "kind": kind, "kernel": k, "ms_median": float(np.median(ts)),
                      "min": float(np.min(ts))}), flush=True)
