#!/usr/bin/env python3
"""Share-envelope kernel rates on one GPU: AES-256-CTR,
encrypt to base64 / to "0x"+hex and back, over a message the size of one
share's packed records at 2^24 elements (1.13 GB), for both LDS table layouts
(DN_AES_TABLES=4 / 2) and store policies (DN_AES_STORE).  HIP events on the launch stream; one JSON line per case.
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "delta-node_amd"), ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)

import torch  # noqa: E402

from delta_node.crypto import aes  # noqa: E402

N = int(os.environ.get("AES_BYTES", "1132427034"))
REPS = 5


def timed(fn):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(REPS):
        out = fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / REPS, out


def main():
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev)
    g.manual_seed(1)
    data = torch.randint(0, 256, (N,), dtype=torch.uint8, device=dev, generator=g)
    key, nonce = bytes(range(32)), bytes(range(16, 32))
    blocks = (N + 15) // 16
    for ntab, store in (("4", "plain"), ("2", "plain"), ("4", "nt")):
        os.environ["DN_AES_TABLES"] = ntab
        os.environ["DN_AES_STORE"] = store
        ms, ct = timed(lambda: aes.ctr_vec(key, nonce, data))
        rows = [("ctr", ms, N + N)]
        del ct
        for hex_ in (False, True):
            ms, text = timed(lambda: aes.encrypt_vec(key, data, nonce=nonce, hex=hex_))
            rows.append(("encrypt_hex" if hex_ else "encrypt_b64", ms, N + text.numel()))
            ms, back = timed(lambda: aes.decrypt_vec(key, text, hex=hex_))
            ok = bool(torch.equal(back, data))
            rows.append(("decrypt_hex" if hex_ else "decrypt_b64", ms, N + text.numel()))
            rows[-1] = rows[-1] + (ok,)
            del text, back
        for r in rows:
            name, ms, hbm = r[:3]
            print(json.dumps({"tables": int(ntab), "store": store, "op": name, "bytes": N, "ms": ms,
                              "plaintext_GBps": N / (ms * 1e-3) / 1e9, "hbm_GBps": hbm / (ms * 1e-3) / 1e9,
                              "lds_lookup_GBps": blocks * 14 * 16 * 4 / (ms * 1e-3) / 1e9,
                              **({"roundtrip_equal": r[3]} if len(r) > 3 else {})}), flush=True)


if __name__ == "__main__":
    main()
