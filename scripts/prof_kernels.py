#!/usr/bin/env python3
"""Profiling driver for rocprofv3 (kernel-trace or PMC passes).

Runs the headline workload's two kernels a few times each on 2^24 elements
(inputs prepared exactly like bench.py) and nothing else on the GPU, so that
per-dispatch counters map 1:1 to split / reconstruct launches.
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "delta-node_amd"))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from delta_node.crypto import shamir  # noqa: E402
from delta_node.crypto.shamir import _native, field, memory  # noqa: E402

reps = int(os.environ.get("REPS", "5"))
log2n = int(os.environ.get("LOG2N", "24"))
N = 1 << log2n
dev = torch.device("cuda", 0)
rng = np.random.default_rng(1)
sec = torch.from_numpy(rng.integers(-(1 << 63), (1 << 63) - 1, size=N, endpoint=True, dtype=np.int64)).to(dev)
ss = shamir.SecretShare(3)
ss.random.seed(1)
coeffs = ss.draw_coeffs_vec(N, dev)
shares = memory.share_block((5, field.vec_bytes(N)), dev)  # as bench.py's blocks
rec = torch.empty(N, dtype=torch.int64, device=dev)
w = _native.lagrange([1, 3, 5], 3)
torch.cuda.synchronize()
for _ in range(reps):
    _native.split_u64(sec, coeffs, shares, N, 3, 5)
for _ in range(reps):
    _native.reconstruct([shares[0], shares[2], shares[4]], w, out_u64=rec, n=N)
torch.cuda.synchronize()
assert torch.equal(rec, sec)
print("ok", reps, "x split + reconstruct of", N)
if os.environ.get("EXTRA", "1") == "1":
    # the fused bit-exact draw + split (make_shares_vec's default: mt_gen_kernel<3>)
    # and the mask row (bounded_acc_kernel, 10 generators, fixed-point base)
    from delta_node.utils import masked_sum  # noqa: E402

    del coeffs
    for i in range(reps):
        ss.make_shares_vec(sec, 5, out=shares)
    val = torch.randn(N, dtype=torch.float64, device=dev)
    terms = [(bytes([i]) * 32, 1 if i % 2 else -1) for i in range(10)]
    out = torch.empty(N, dtype=torch.int64, device=dev)
    for _ in range(reps):
        masked_sum(val, terms, precision=8, out=out)
    torch.cuda.synchronize()
    print("ok", reps, "x fused draw+split and mask row of", N)
