#!/usr/bin/env python3
"""Split duration as a function of the kernel launched before it (one process).

Each variant runs [pre(); split()] x ITERS and times only the split launches
with HIP events on the launch stream.  Prints one JSON line per variant."""
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
ITERS = int(os.environ.get("ITERS", "15"))
dev = torch.device("cuda", 0)
rng = np.random.default_rng(1)
sec = torch.from_numpy(rng.integers(-(1 << 63), (1 << 63) - 1, size=N, endpoint=True, dtype=np.int64)).to(dev)
ss = shamir.SecretShare(3)
ss.random.seed(1)
coeffs = ss.draw_coeffs_vec(N, dev)
shares = torch.empty((5, field.vec_bytes(N)), dtype=torch.uint8, device=dev)
rec = torch.empty(N, dtype=torch.int64, device=dev)
rec_fe = torch.empty(field.vec_bytes(N), dtype=torch.uint8, device=dev)
scratch = torch.empty(3 * field.vec_bytes(N) // 8, dtype=torch.int64, device=dev)
w135 = _native.lagrange([1, 3, 5], 3)
rows = [shares[0], shares[2], shares[4]]
stream = torch.cuda.current_stream()


def split():
    _native.split_u64(sec, coeffs, shares, N, 3, 5)


def recon():
    _native.reconstruct(rows, w135, out_u64=rec, n=N)


def recon_fe():
    _native.reconstruct(rows, w135, out_fe=rec_fe, n=N)


def recon_noroll():
    os.environ["DN_RECON_UNROLL"] = "0"
    _native.reconstruct(rows, w135, out_u64=rec, n=N)
    os.environ.pop("DN_RECON_UNROLL")


variants = {
    "none": lambda: None,
    "reconstruct_u64": recon,
    "reconstruct_fe": recon_fe,
    "reconstruct_noroll": recon_noroll,
    "fill_rec_128MB": lambda: rec.fill_(7),
    "fill_scratch_3GB": lambda: scratch.fill_(7),
    "read_shares_3rows": lambda: torch.sum(shares[0:5:2].view(torch.int64), dtype=torch.int64),
    "sleep_600us": lambda: torch.cuda._sleep(1_500_000),
    "split": split,
}
order = os.environ.get("VARIANTS", ",".join(variants)).split(",")
res = {}
for rnd in range(3):
    for name in order:
        pre = variants[name]
        for _ in range(2):
            pre()
            split()
        evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(ITERS)]
        torch.cuda.synchronize()
        for s, e in evs:
            pre()
            s.record(stream)
            split()
            e.record(stream)
        torch.cuda.synchronize()
        res.setdefault(name, []).extend(s.elapsed_time(e) for s, e in evs)
for name in order:
    ts = np.array(res[name])
    print(json.dumps({"pre": name, "split_ms_median": float(np.median(ts)), "min": float(ts.min()),
                      "max": float(ts.max())}), flush=True)
