#!/usr/bin/env python3
"""Why the bench's PRNG row reads slower than scripts/prng_ab.py: the same
ChaCha20 / 8 split (3-of-5, 2^24) timed the bench's way (mean of 5 after one
warm-up call) with the bench's secrets (bench.secrets_int64: full int64 range)
and with prng_ab's (torch.randint in +-2^62), in both orders.  One JSON line."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "delta-node_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402
from delta_node.crypto.shamir import _native, field  # noqa: E402

n = 1 << 24
dev = torch.device("cuda", 0)
sh = torch.empty((5, field.vec_bytes(n)), dtype=torch.uint8, device=dev)
secs = {"bench_full_int64": torch.from_numpy(bench.secrets_int64(3, n)).to(dev),
        "randint_2e62": torch.randint(-(1 << 62), 1 << 62, (n,), dtype=torch.int64, device=dev)}


def mean5(sec, rounds):
    _native.split_prng(sec, bytes(range(32)), 0, rounds, 0, sh, n, 3, 5)
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(5):
        _native.split_prng(sec, bytes(range(32)), 0, rounds, 0, sh, n, 3, 5)
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / 5


res = {}
for rep in range(2):
    for name, sec in secs.items():
        for rounds in (20, 8):
            res[f"{name}_chacha{rounds}_rep{rep}"] = mean5(sec, rounds)
print(json.dumps(res))
