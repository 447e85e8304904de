#!/usr/bin/env python3
"""Split duration per share allocation for share-store cache policies
(DN_STORE_AUX = 0 / 1 / 2 (default, nt) / 3), interleaved in one process."""
import json
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
stream = torch.cuda.current_stream()
AUX = os.environ.get("AUXES", "2,0,1,3").split(",")


def timed(fn, iters=8):
    fn()
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(iters)]
    for a, b in evs:
        a.record(stream)
        fn()
        b.record(stream)
    torch.cuda.synchronize()
    return [a.elapsed_time(b) for a, b in evs]


res = {}
ref = None
for rnd in range(3):
    for i, sh in enumerate(sets):
        for aux in AUX:
            os.environ["DN_STORE_AUX"] = aux
            res.setdefault((i, aux), []).extend(timed(lambda: _native.split_u64(sec, coeffs, sh, N, 3, 5)))
            if ref is None:
                ref = sh[:, :1 << 20].clone()
            assert torch.equal(sh[:, :1 << 20], ref)
for (i, aux), ts in sorted(res.items()):
    print(json.dumps({"set": i, "store_aux": aux, "ms_median": float(np.median(ts)), "min": float(np.min(ts))}),
          flush=True)
