#!/usr/bin/env python3
"""The share-envelope encrypt kernel alone (dn_aes_encrypt to hex, 1.13 GB of
records, preallocated output), HIP events on its stream, best of 3 rounds of
5 launches, under the library DN_SHAMIR_LIB selects (A/B of variants).
One JSON line."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "delta-node_amd"))

import torch  # noqa: E402

from delta_node.crypto.aes import aes as aes_mod  # noqa: E402
from delta_node.crypto.shamir import _native  # noqa: E402

N = int(os.environ.get("AES_BYTES", "1132427034"))
dev = torch.device("cuda", 0)
g = torch.Generator(device=dev)
g.manual_seed(1)
data = torch.randint(0, 256, (N,), dtype=torch.uint8, device=dev, generator=g)
key, nonce = bytes(range(32)), bytes(range(16, 32))
AL = aes_mod._lib()
out = torch.empty(int(AL.dn_aes_encrypt_len(N, 1)), dtype=torch.uint8, device=dev)
stream = torch.cuda.current_stream()


def k():
    _native.check(AL.dn_aes_encrypt(key, len(key), nonce, data.data_ptr(), N, out.data_ptr(), 1, stream.cuda_stream))


for _ in range(3):
    k()
best = None
for _ in range(3):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record(stream)
    for _ in range(5):
        k()
    e.record(stream)
    e.synchronize()
    ms = s.elapsed_time(e) / 5
    best = ms if best is None else min(best, ms)
lds = (N + 15) // 16 * 14 * 16 * 4
# the receiver's side: dn_aes_decrypt of the same text as the JSON carries it
# (after "0x": 2 bytes into an aligned buffer), into a preallocated output
import ctypes  # noqa: E402

L = out.numel()
text = torch.empty(L + 16, dtype=torch.uint8, device=dev)
text[2:2 + L].copy_(out)
cap = int(AL.dn_aes_decrypt_capacity(L, 1))
back = torch.empty(cap + 16, dtype=torch.uint8, device=dev)
olen = torch.zeros(1, dtype=torch.int64, device=dev)
bad = torch.zeros(1, dtype=torch.int32, device=dev)


def d():
    _native.check(AL.dn_aes_decrypt(key, len(key), text.data_ptr() + 2, L, 1, back.data_ptr(), cap + 16,
                                    olen.data_ptr(), bad.data_ptr(), stream.cuda_stream))


for _ in range(3):
    d()
dbest = None
for _ in range(3):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record(stream)
    for _ in range(5):
        d()
    e.record(stream)
    e.synchronize()
    ms = s.elapsed_time(e) / 5
    dbest = ms if dbest is None else min(dbest, ms)
ok = bool(torch.equal(back[:N], data)) and int(olen.item()) == N and int(bad.item()) == 0
print(json.dumps({"lib": os.path.basename(_native.lib_path()), "encrypt_hex_kernel_ms": best,
                  "lds_frac": lds / (best * 1e-3) / 75e12, "decrypt_hex_kernel_ms": dbest,
                  "decrypt_lds_frac": lds / (dbest * 1e-3) / 75e12, "roundtrip": ok,
                  "digest": int(out[:1 << 20].sum().item())}))
