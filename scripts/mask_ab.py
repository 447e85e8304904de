#!/usr/bin/env python3
"""A/B of the mask accumulate kernel (dn_bounded_i64_accumulate, SURVEY §8(f)
row 1) between library builds: the bench row's workload — fix_precision of
2^24 float64 + 10 signed make_mask generators, one launch — timed with events
on the launch stream (best of 3 rounds of 5 launches), the output's SHA-256
and a 2^14 prefix against numpy (the reference's generator).  The library is
DN_SHAMIR_LIB (default: the product build).  Prints one JSON line."""
import hashlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "delta-node_amd"))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from delta_node.crypto.shamir import _native  # noqa: E402
from delta_node.utils import _mask_native as mn  # noqa: E402
from oracle import py_mask as pm  # noqa: E402


def main() -> int:
    log2n = int(os.environ.get("LOG2N", "24"))
    n = 1 << log2n
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev)
    g.manual_seed(3)
    val = torch.randn(n, dtype=torch.float64, device=dev, generator=g) * 1e3
    seeds = [bytes([7 * i + j for j in range(32)]) for i in range(10)]
    signs = [1] + [(-1) ** i for i in range(9)]
    gens = [mn.pcg64(sd) for sd in seeds]
    out = torch.empty(n, dtype=torch.int64, device=dev)
    flags = torch.zeros(len(gens), dtype=torch.int32, device=dev)
    stream = torch.cuda.current_stream()
    for _ in range(3):
        mn.accumulate(gens, signs, out, n, 0, 2 ** 47 - 2, base_f64=val, precision=8, rejects=flags)
    torch.cuda.synchronize()
    best = []
    for _ in range(3):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record(stream)
        for _ in range(5):
            mn.accumulate(gens, signs, out, n, 0, 2 ** 47 - 2, base_f64=val, precision=8, rejects=flags)
        e.record(stream)
        torch.cuda.synchronize()
        best.append(s.elapsed_time(e) / 5)
    k = 1 << 14
    want = pm.fix_precision(val[:k].cpu().numpy(), 8)
    for sd, sg in zip(seeds, signs):
        want = want + sg * pm.make_mask_numpy(sd, (k,))
    ok = bool(np.array_equal(out[:k].cpu().numpy(), want))
    digest = hashlib.sha256(out.cpu().numpy().tobytes()).hexdigest()[:16]
    ms = min(best)
    mix = 1.0 / (23.5 / 3.6e13 + 22.0 / 6.1e13)
    print(json.dumps({"lib": os.path.basename(_native.lib_path()), "log2n": log2n, "kernel_ms": ms, "rounds_ms": best,
                      "draws_per_s": 10 * n / (ms * 1e-3), "mix_bound_frac": 10 * n / (ms * 1e-3) / mix,
                      "numpy_prefix_equal": ok, "digest": digest, "rejects": int(flags.sum().item())}), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
