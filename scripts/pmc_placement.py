#!/usr/bin/env python3
"""Workload for the placement PMC passes: split 3-of-5 at 2^24 into SETS fresh
share allocations, REPS launches each (dispatch order = set-major)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "delta-node_amd"))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from delta_node.crypto import shamir  # noqa: E402
from delta_node.crypto.shamir import _native, field  # noqa: E402

N = 1 << 24
dev = torch.device("cuda", 0)
rng = np.random.default_rng(1)
sec = torch.from_numpy(rng.integers(-(1 << 63), (1 << 63) - 1, size=N, endpoint=True, dtype=np.int64)).to(dev)
ss = shamir.SecretShare(3)
ss.random.seed(1)
coeffs = ss.draw_coeffs_vec(N, dev)
sets = [torch.empty((5, field.vec_bytes(N)), dtype=torch.uint8, device=dev) for _ in range(int(os.environ.get("SETS", "6")))]
for sh in sets:
    for _ in range(int(os.environ.get("REPS", "3"))):
        _native.split_u64(sec, coeffs, sh, N, 3, 5)
torch.cuda.synchronize()
