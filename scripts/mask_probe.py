#!/usr/bin/env python3
"""Mask row A/B: masked_sum over 10 generators at 2^24 (bench.py mask_row's
workload) with the product library and with tuning-library variants
(MASK_VARIANTS="DN_MASK_SB=1;..."); one JSON line."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "delta-node_amd"), ROOT]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from delta_node.crypto.shamir import _native  # noqa: E402
from delta_node.utils import masked_sum  # noqa: E402
from oracle import py_mask as pm  # noqa: E402

dev = torch.device("cuda", 0)
n = 1 << int(os.environ.get("LOG2N", "24"))
val = torch.randn(n, dtype=torch.float64, device=dev) * 1e3
rng = np.random.default_rng(1)
terms = [(bytes(rng.integers(0, 256, 32, dtype=np.uint8)), 1)] + \
        [(bytes(rng.integers(0, 256, 32, dtype=np.uint8)), (-1) ** i) for i in range(9)]
k = 1 << 14
want = pm.fix_precision(val[:k].cpu().numpy(), 8)
for sd, sg in terms:
    want = want + sg * pm.make_mask_numpy(sd, (k,))


def timed(reps=10):
    out = torch.empty(n, dtype=torch.int64, device=dev)
    masked_sum(val, terms, precision=8, out=out)
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        masked_sum(val, terms, precision=8, out=out)
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps, bool(np.array_equal(out[:k].cpu().numpy(), want))


variants = [v for v in os.environ.get("MASK_VARIANTS", "DN_MASK_SB=1").split(";") if v]
rounds = int(os.environ.get("ROUNDS", "3"))
times = {"product": []}
for _ in range(rounds):  # alternate product and variants, keep every sample (placement / clock noise)
    times["product"].append(timed())
    for var in variants:
        kv = dict(x.split("=") for x in var.split(","))
        os.environ.update(kv)
        with _native.library(_native.TUNING_LIB):
            times.setdefault(var, []).append(timed())
        for kk in kv:
            del os.environ[kk]
out = {}
for kk, v in times.items():
    ms = sorted(x[0] for x in v)
    out[kk] = {"ms_median": ms[len(ms) // 2], "ms_all": ms, "draws_per_s": 10 * n / (ms[len(ms) // 2] * 1e-3),
               "numpy_prefix_equal": all(x[1] for x in v)}
print(json.dumps(out))
