#!/usr/bin/env python3
"""Profiling driver: make_shares_vec(2^24 int64, 5) with the default (fused
MT19937 draw + split, mt_gen_kernel<3>) REPS times, nothing else timed."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "delta-node_amd"), ROOT]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from delta_node.crypto import shamir  # noqa: E402
from delta_node.crypto.shamir import field  # noqa: E402

N = 1 << int(os.environ.get("LOG2N", "24"))
dev = torch.device("cuda", 0)
sec = torch.from_numpy(np.random.default_rng(1).integers(-(1 << 62), 1 << 62, N, dtype=np.int64)).to(dev)
out = torch.empty((5, field.vec_bytes(N)), dtype=torch.uint8, device=dev)
ss = shamir.SecretShare(3)
ss.random.seed(1)
for _ in range(int(os.environ.get("REPS", "3"))):
    ss.make_shares_vec(sec, 5, out=out)
torch.cuda.synchronize()
print("ok")
