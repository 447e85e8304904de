#!/usr/bin/env python3
"""Split duration vs where its buffers live (one process, interleaved rounds).

Sets: two independent torch allocations, one carved torch arena, per-buffer
hipMalloc, and hipExtMallocWithFlags(hipDeviceMallocContiguous).  Same data in
every set; only the split launches are timed (HIP events, launch stream)."""
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
sec0 = torch.from_numpy(rng.integers(-(1 << 63), (1 << 63) - 1, size=N, endpoint=True, dtype=np.int64)).to(dev)
ss = shamir.SecretShare(3)
ss.random.seed(1)
coeffs0 = ss.draw_coeffs_vec(N, dev)
hip = ctypes.CDLL("libamdhip64.so")


class Raw:
    def __init__(self, p):
        self.p = p

    def data_ptr(self):
        return self.p


def hip_alloc(nbytes, flags=None):
    p = ctypes.c_void_p()
    rc = hip.hipExtMallocWithFlags(ctypes.byref(p), ctypes.c_size_t(nbytes), flags) if flags is not None \
        else hip.hipMalloc(ctypes.byref(p), ctypes.c_size_t(nbytes))
    if rc != 0:
        raise RuntimeError(f"hip alloc rc={rc}")
    return p.value


def fill(dst_ptr, src):
    torch.cuda.synchronize()
    hip.hipMemcpy(ctypes.c_void_p(dst_ptr), ctypes.c_void_p(src.data_ptr()), ctypes.c_size_t(src.numel() * src.element_size()), 3)


sets = {}
for name in ("torch_a", "torch_b"):
    s = torch.empty_like(sec0).copy_(sec0)
    c = torch.empty_like(coeffs0).copy_(coeffs0)
    sh = torch.empty((5, VB), dtype=torch.uint8, device=dev)
    sets[name] = (s, c, sh)
align = 1 << 21
sizes = [sec0.numel() * 8, coeffs0.numel(), 5 * VB]
offs, tot = [], 0
for b in sizes:
    offs.append(tot)
    tot += -(-b // align) * align
arena = torch.empty(tot + align, dtype=torch.uint8, device=dev)
base = -(-arena.data_ptr() // align) * align
sets["arena"] = tuple(Raw(base + o) for o in offs)
fill(sets["arena"][0].p, sec0)
fill(sets["arena"][1].p, coeffs0)
for name, flags in (("hipMalloc", None), ("hip_contig", 4)):
    try:
        ps = [hip_alloc(b, flags) for b in sizes]
    except RuntimeError as e:
        print(json.dumps({"set": name, "error": str(e)}), flush=True)
        continue
    sets[name] = tuple(Raw(p) for p in ps)
    fill(ps[0], sec0)
    fill(ps[1], coeffs0)
if os.environ.get("FACTORIAL") and "hipMalloc" in sets:
    import itertools

    pools = {"T": sets["torch_a"], "H": sets["hipMalloc"]}
    sets = {"".join(k): tuple(pools[k[i]][i] for i in range(3)) for k in itertools.product("TH", repeat=3)}
torch.cuda.synchronize()
stream = torch.cuda.current_stream()
res = {}
for rnd in range(4):
    for name, (s, c, sh) in sets.items():
        _native.split_u64(s, c, sh, N, 3, 5)
        evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(10)]
        for a, b in evs:
            a.record(stream)
            _native.split_u64(s, c, sh, N, 3, 5)
            b.record(stream)
        torch.cuda.synchronize()
        res.setdefault(name, []).extend(a.elapsed_time(b) for a, b in evs)
ref = None
for name, (s, c, sh) in sets.items():
    ts = np.array(res[name])
    head = np.empty(4096, dtype=np.uint8)
    hip.hipMemcpy(ctypes.c_void_p(head.ctypes.data), ctypes.c_void_p(sh.data_ptr() + 2 * VB), ctypes.c_size_t(4096), 2)
    ref = head if ref is None else ref
    print(json.dumps({"set": name, "split_ms_median": float(np.median(ts)), "min": float(ts.min()),
                      "max": float(ts.max()), "same_output": bool(np.array_equal(head, ref)),
                      "ptrs": [hex(x.data_ptr()) for x in (s, c, sh)]}), flush=True)
