#!/usr/bin/env python3
"""Fixed cost of make_shares_vec's fused MT19937 draw + split (the drop-in
vector path) per call: wall time per call at several sizes, 3-of-5, shares
preallocated.  Prints one JSON line."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "delta-node_amd"))

import torch  # noqa: E402

from delta_node.crypto import shamir  # noqa: E402
from delta_node.crypto.shamir import field  # noqa: E402

dev = torch.device("cuda", 0)
out = {}
for lg in (8, 12, 16, 20, 24):
    N = 1 << lg
    sec = torch.randint(-(1 << 62), 1 << 62, (N,), dtype=torch.int64, device=dev)
    sh = torch.empty((5, field.vec_bytes(N)), dtype=torch.uint8, device=dev)
    ss = shamir.SecretShare(3)
    ss.random.seed(lg)
    for _ in range(3):
        ss.make_shares_vec(sec, 5, out=sh)
    torch.cuda.synchronize()
    reps = 50 if lg < 24 else 10
    t0 = time.perf_counter()
    for _ in range(reps):
        ss.make_shares_vec(sec, 5, out=sh)
    torch.cuda.synchronize()
    out[f"2^{lg}"] = (time.perf_counter() - t0) / reps * 1e3
# the product default: out=None (each call's share block from memory.share_block;
# the previous call's block returns to the pool when its tensor is dropped)
dflt = {}
for lg in (20, 24):
    N = 1 << lg
    sec = torch.randint(-(1 << 62), 1 << 62, (N,), dtype=torch.int64, device=dev)
    ss = shamir.SecretShare(3)
    ss.random.seed(lg)
    for _ in range(3):
        sh = ss.make_shares_vec(sec, 5)
        del sh
    torch.cuda.synchronize()
    reps = 50 if lg < 24 else 10
    t0 = time.perf_counter()
    for _ in range(reps):
        sh = ss.make_shares_vec(sec, 5)
        del sh
    torch.cuda.synchronize()
    dflt[f"2^{lg}"] = (time.perf_counter() - t0) / reps * 1e3
print(json.dumps({"make_shares_vec_ms_per_call": out, "make_shares_vec_default_out_ms_per_call": dflt}))

# the same 2^12 call through the C-ABI directly (arguments prepared once):
# the difference to make_shares_vec is the binding's Python time per call
from delta_node.crypto.shamir import _native  # noqa: E402

N = 1 << 12
sec = torch.randint(-(1 << 62), 1 << 62, (N,), dtype=torch.int64, device=dev)
sh = torch.empty((5, field.vec_bytes(N)), dtype=torch.uint8, device=dev)
ss = shamir.SecretShare(3)
ss.random.seed(12)
L = _native.lib()
sb = int(L.dn_mt19937_device_scratch_bytes(N, 2))
scratch = torch.empty(sb, dtype=torch.uint8, device=dev)
ip = _native._mt_inplace(ss.random)
args = (ip[0], ip[1], sec.data_ptr(), sh.data_ptr(), N, 3, 5, scratch.data_ptr(), sb, _native.stream_ptr())
for _ in range(5):
    assert L.dn_mt19937_split_device(*args) == 0
reps = 200
t0 = time.perf_counter()
for _ in range(reps):
    L.dn_mt19937_split_device(*args)
raw = (time.perf_counter() - t0) / reps * 1e3
t0 = time.perf_counter()
for _ in range(reps):
    ss.make_shares_vec(sec, 5, out=sh)
api = (time.perf_counter() - t0) / reps * 1e3
print(json.dumps({"2^12_raw_c_abi_ms": raw, "2^12_make_shares_vec_ms": api}))
