#!/usr/bin/env python3
"""Does the ChaCha20 split slow down after sustained load (power / clock)?
ChaCha20 / 8 split times (3-of-5, 2^24, best of 3 rounds of 5) cold, then
again right after ~3 s of AES-envelope encrypt launches (the work the bench
runs before its PRNG row), then after 2 s idle.  Prints one JSON line."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "delta-node_amd"))

import torch  # noqa: E402

from delta_node.crypto import aes  # noqa: E402
from delta_node.crypto.shamir import _native, field  # noqa: E402

n = 1 << 24
dev = torch.device("cuda", 0)
sec = torch.randint(-(1 << 62), 1 << 62, (n,), dtype=torch.int64, device=dev)
sh = torch.empty((5, field.vec_bytes(n)), dtype=torch.uint8, device=dev)
data = torch.randint(0, 256, (1132427034,), dtype=torch.uint8, device=dev)


def prng(rounds):
    best = None
    for _ in range(3):
        _native.split_prng(sec, bytes(range(32)), 0, rounds, 0, sh, n, 3, 5)
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(5):
            _native.split_prng(sec, bytes(range(32)), 0, rounds, 0, sh, n, 3, 5)
        e.record()
        torch.cuda.synchronize()
        ms = s.elapsed_time(e) / 5
        best = ms if best is None else min(best, ms)
    return best


res = {"cold": {"chacha20_ms": prng(20), "chacha8_ms": prng(8)}}
t0 = time.time()
k = 0
while time.time() - t0 < 3.0:
    aes.encrypt_vec(bytes(range(32)), data, nonce=bytes(16), hex=True)
    k += 1
    if k % 8 == 0:
        torch.cuda.synchronize()
res["after_aes"] = {"chacha20_ms": prng(20), "chacha8_ms": prng(8), "aes_calls": k}
time.sleep(2.0)
res["after_idle"] = {"chacha20_ms": prng(20), "chacha8_ms": prng(8)}
t0 = time.time()
while time.time() - t0 < 3.0:
    _native.split_prng(sec, bytes(range(32)), 0, 20, 0, sh, n, 3, 5)
    torch.cuda.synchronize()
res["after_prng20_3s"] = {"chacha20_ms": prng(20), "chacha8_ms": prng(8)}
print(json.dumps(res))
