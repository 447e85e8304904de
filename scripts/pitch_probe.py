#!/usr/bin/env python3
"""Split duration vs share/coefficient row pitch (vec_bytes + pad), for torch
and physically contiguous allocations.  Tests whether rows a multiple of 2^25
bytes apart alias in DRAM.  One JSON line per (alloc, pad)."""
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
coeffs0 = ss.draw_coeffs_vec(N, dev)
hip = ctypes.CDLL("libamdhip64.so")
PADS = [int(x) for x in os.environ.get("PADS", "0,256,4096,16896,65536,1048576,2097152,6291456").split(",")]


class Raw:
    def __init__(self, p):
        self.p = p

    def data_ptr(self):
        return self.p


def alloc(kind, nbytes):
    if kind == "torch":
        t = torch.empty(nbytes, dtype=torch.uint8, device=dev)
        return t, t.data_ptr()
    p = ctypes.c_void_p()
    if hip.hipExtMallocWithFlags(ctypes.byref(p), ctypes.c_size_t(nbytes), 4) != 0:
        raise RuntimeError("hipExtMallocWithFlags failed")
    return None, p.value


def d2d(dst, src, nbytes):
    hip.hipMemcpy(ctypes.c_void_p(dst), ctypes.c_void_p(src), ctypes.c_size_t(nbytes), 3)


sets = {}
for kind in os.environ.get("KINDS", "torch,contig").split(","):
    for pad in PADS:
        pitch = VB + pad
        hc, pc = alloc(kind, 2 * pitch)
        hs, ps = alloc(kind, 5 * pitch)
        torch.cuda.synchronize()
        for j in range(2):
            d2d(pc + j * pitch, coeffs0[j].data_ptr(), VB)
        sets[(kind, pad)] = (Raw(pc), Raw(ps), pitch, hc, hs)
torch.cuda.synchronize()
stream = torch.cuda.current_stream()
res = {}
for rnd in range(3):
    for (kind, pad), (c, sh, pitch, _, _) in sets.items():
        os.environ["DN_ROW_PAD"] = str(pad)
        _native.split_u64(sec, c, sh, N, 3, 5)
        evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(8)]
        for a, b in evs:
            a.record(stream)
            _native.split_u64(sec, c, sh, N, 3, 5)
            b.record(stream)
        torch.cuda.synchronize()
        res.setdefault((kind, pad), []).extend(a.elapsed_time(b) for a, b in evs)
os.environ.pop("DN_ROW_PAD", None)
ref = None
for (kind, pad), (c, sh, pitch, _, _) in sets.items():
    ts = np.array(res[(kind, pad)])
    tail = np.empty(4096, dtype=np.uint8)
    hip.hipMemcpy(ctypes.c_void_p(tail.ctypes.data), ctypes.c_void_p(sh.p + 4 * pitch + VB - 4096), ctypes.c_size_t(4096), 2)
    ref = tail if ref is None else ref
    print(json.dumps({"alloc": kind, "pad": pad, "split_ms_median": float(np.median(ts)), "min": float(ts.min()),
                      "max": float(ts.max()), "same_output": bool(np.array_equal(tail, ref)),
                      "shares_ptr": hex(sh.p)}), flush=True)
