#!/usr/bin/env python3
"""Share-envelope kernel times of one library (DN_SHAMIR_LIB selects it):
AES-256-CTR, encrypt to base64 / "0x"+hex and decrypt back, over the packed
records of one share at 2^24 elements (1.13 GB).  HIP events on the launch
stream, best of 3 rounds of 5 launches.  Prints one JSON line."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "delta-node_amd"))

import torch  # noqa: E402

from delta_node.crypto import aes  # noqa: E402

N = 1132427034
dev = torch.device("cuda", 0)
g = torch.Generator(device=dev)
g.manual_seed(1)
data = torch.randint(0, 256, (N,), dtype=torch.uint8, device=dev, generator=g)
key, nonce = bytes(range(32)), bytes(range(16, 32))


def timed(fn, reps=5):
    best = None
    for _ in range(3):
        fn()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(reps):
            out = fn()
        e.record()
        torch.cuda.synchronize()
        ms = s.elapsed_time(e) / reps
        best = ms if best is None else min(best, ms)
    return best, out


res = {"lib": os.path.basename(os.environ.get("DN_SHAMIR_LIB", "libdn_shamir.so"))}
res["ctr_ms"], ct = timed(lambda: aes.ctr_vec(key, nonce, data))
del ct
for hex_ in (False, True):
    tag = "hex" if hex_ else "b64"
    res[f"encrypt_{tag}_ms"], text = timed(lambda: aes.encrypt_vec(key, data, nonce=nonce, hex=hex_))
    res[f"decrypt_{tag}_ms"], back = timed(lambda: aes.decrypt_vec(key, text, hex=hex_))
    res[f"roundtrip_{tag}"] = bool(torch.equal(back, data))
    del text, back
lds_bytes = (N + 15) // 16 * 14 * 16 * 4
res["encrypt_hex_lds_frac"] = lds_bytes / (res["encrypt_hex_ms"] * 1e-3) / 75e12
res["ctr_lds_frac"] = lds_bytes / (res["ctr_ms"] * 1e-3) / 75e12
print(json.dumps(res))
