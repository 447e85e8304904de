#!/usr/bin/env python3
"""Host-memory (PCIe-inclusive) rate of the split path, for DESIGN.md §7.

The reference path starts with the result tensor in host memory and ends with
serialized shares handed to the HTTP peer.  Measured here, for 2^24 int64
elements, 3-of-5:

  A  drop-in call: make_shares_vec(host int64) -> MT19937 coefficient draw on the
     host + H2D + split; then D2H of the 5 share vectors into pinned memory.
  B  pipelined: 2^20-element chunks; the host draws chunk c+1's coefficients
     while the GPU copies/splits/copies back chunk c (two streams).
  C  transfer ceilings: pinned H2D and D2H bandwidth alone.
  D  device-PRNG drop-in: make_shares_vec_prng(host int64) -> H2D of the
     secrets + split with ChaCha20 coefficients on the GPU, then D2H of the
     shares (no host coefficient draw, no coefficient transfer).
  E  the bit-exact drop-in as shipped: make_shares_vec(host int64) with the
     reference's MT19937 coefficients drawn on the GPU (jump-ahead
     substreams, dn_mt19937_draw_coeffs_device), then D2H; the shares equal
     A's byte for byte.

Prints one JSON object.
"""
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "delta-node_amd"))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from delta_node.crypto import shamir  # noqa: E402
from delta_node.crypto.shamir import _native, field  # noqa: E402

N = 1 << int(os.environ.get("LOG2N", "24"))
T, NS = 3, 5
dev = torch.device("cuda", 0)
rng = np.random.default_rng(1)
sec_h = rng.integers(-(1 << 63), (1 << 63) - 1, size=N, endpoint=True, dtype=np.int64)
out = {"N": N, "t": T, "n": NS}


def sync():
    torch.cuda.synchronize()


# ---- C: transfer ceilings -------------------------------------------------
big = torch.empty(1 << 30, dtype=torch.uint8, pin_memory=True)
dbig = torch.empty(1 << 30, dtype=torch.uint8, device=dev)
dbig.copy_(big, non_blocking=True)
sync()
t0 = time.perf_counter()
for _ in range(3):
    dbig.copy_(big, non_blocking=True)
sync()
out["h2d_pinned_GBps"] = 3 * big.numel() / (time.perf_counter() - t0) / 1e9
t0 = time.perf_counter()
for _ in range(3):
    big.copy_(dbig, non_blocking=True)
sync()
out["d2h_pinned_GBps"] = 3 * big.numel() / (time.perf_counter() - t0) / 1e9
del big, dbig

# ---- A: drop-in call, phase by phase --------------------------------------
ss = shamir.SecretShare(T)
ss.random.seed(1)
vb = field.vec_bytes(N)
host_shares = torch.empty((NS, vb), dtype=torch.uint8, pin_memory=True)
sync()
t0 = time.perf_counter()
host_coeffs = _native.mt_draw_coeffs(ss.random, N, T - 1)
t1 = time.perf_counter()
coeffs = torch.from_numpy(host_coeffs).to(dev)
sec = torch.from_numpy(sec_h).to(dev)
sync()
t2 = time.perf_counter()
shares = ss.make_shares_vec(sec, NS, coeffs=coeffs)
sync()
t3 = time.perf_counter()
host_shares.copy_(shares)
sync()
t4 = time.perf_counter()
host_shares_a = host_shares.clone()
out["A_dropin"] = {"mt_draw_s": t1 - t0, "h2d_s": t2 - t1, "split_s": t3 - t2, "d2h_s": t4 - t3,
                   "total_s": t4 - t0, "elems_per_s": N / (t4 - t0), "input_MBps": N * 8 / (t4 - t0) / 1e6}
del coeffs, shares

# ---- B: pipelined chunks ---------------------------------------------------
C = 1 << 20
nch = N // C
vbc = field.vec_bytes(C)
ss.random.seed(1)
streams = [torch.cuda.Stream(), torch.cuda.Stream()]
bufs = [{"sec": torch.empty(C, dtype=torch.int64, device=dev),
         "co": torch.empty((T - 1, vbc), dtype=torch.uint8, device=dev),
         "sh": torch.empty((NS, vbc), dtype=torch.uint8, device=dev)} for _ in range(2)]
pin_co = [torch.empty((T - 1, vbc), dtype=torch.uint8, pin_memory=True) for _ in range(2)]
pin_sec = torch.from_numpy(sec_h).pin_memory()
pin_out = torch.empty((nch, NS, vbc), dtype=torch.uint8, pin_memory=True)
events = [torch.cuda.Event(), torch.cuda.Event()]
draws = [None] * nch
ready = [threading.Event() for _ in range(nch)]


def producer():
    for c in range(nch):
        draws[c] = _native.mt_draw_coeffs(ss.random, C, T - 1)
        ready[c].set()


sync()
t0 = time.perf_counter()
th = threading.Thread(target=producer)
th.start()
for c in range(nch):
    i = c % 2
    ready[c].wait()
    events[i].synchronize()  # buffer i free again (its previous D2H finished)
    pin_co[i].numpy()[...] = draws[c]
    draws[c] = None
    with torch.cuda.stream(streams[i]):
        b = bufs[i]
        b["sec"].copy_(pin_sec[c * C:(c + 1) * C], non_blocking=True)
        b["co"].copy_(pin_co[i], non_blocking=True)
        _native.split_u64(b["sec"], b["co"], b["sh"], C, T, NS)
        pin_out[c].copy_(b["sh"], non_blocking=True)
        events[i].record(streams[i])
th.join()
sync()
tB = time.perf_counter() - t0
out["B_pipelined"] = {"chunk": C, "total_s": tB, "elems_per_s": N / tB, "input_MBps": N * 8 / tB / 1e6}

# parity of B vs A (same MT stream, chunked): shares equal after re-tiling
a0 = field.vec_to_limbs(host_shares[0].numpy(), N)
b0 = np.concatenate([field.vec_to_limbs(pin_out[c, 0].numpy(), C) for c in range(nch)])
out["B_equals_A"] = bool(np.array_equal(a0, b0))

# ---- D: device-PRNG drop-in -------------------------------------------------
del pin_out, bufs
key = bytes(range(32))
ss.make_shares_vec_prng(torch.from_numpy(sec_h[:4096]), NS, key=key)  # warm the kernel
sync()
t0 = time.perf_counter()
sec = torch.from_numpy(sec_h).to(dev)
sync()
t1 = time.perf_counter()
shares, _ = ss.make_shares_vec_prng(sec, NS, key=key)
sync()
t2 = time.perf_counter()
host_shares.copy_(shares)
sync()
t3 = time.perf_counter()
out["D_prng_dropin"] = {"h2d_s": t1 - t0, "split_s": t2 - t1, "d2h_s": t3 - t2, "total_s": t3 - t0,
                        "elems_per_s": N / (t3 - t0), "input_MBps": N * 8 / (t3 - t0) / 1e6,
                        "roundtrip_equal": bool(torch.equal(
                            ss.resolve_shares_vec([shares[0], shares[2], shares[4]], [1, 3, 5], N), sec))}

# ---- E: bit-exact drop-in, MT19937 drawn on the device ----------------------
ss.random.seed(1)
sync()
t0 = time.perf_counter()
sec = torch.from_numpy(sec_h).to(dev)
sync()
t1 = time.perf_counter()
coeffs = ss.draw_coeffs_vec(N, dev)
sync()
t2 = time.perf_counter()
shares = ss.make_shares_vec(sec, NS, coeffs=coeffs)
sync()
t3 = time.perf_counter()
e_shares = torch.empty((NS, vb), dtype=torch.uint8, pin_memory=True)
t3b = time.perf_counter()
e_shares.copy_(shares)
sync()
t4 = time.perf_counter()
out["E_mt_device_dropin"] = {"h2d_s": t1 - t0, "mt_draw_device_s": t2 - t1, "split_s": t3 - t2,
                             "d2h_s": t4 - t3b, "total_s": (t4 - t3b) + (t3 - t0),
                             "elems_per_s": N / ((t4 - t3b) + (t3 - t0)),
                             "input_MBps": N * 8 / ((t4 - t3b) + (t3 - t0)) / 1e6,
                             "equals_A": bool(torch.equal(e_shares, host_shares_a))}
print(json.dumps(out))
