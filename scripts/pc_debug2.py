#!/usr/bin/env python3
"""Debug: fused draw + split (3-of-5) for substream 0 inside the caller's
array, two-wave vs one-wave kernel (tuning library, DN_MT_PC_FORCE), against
host draw + split: differing elements per share row."""
import json
import os
import random
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "delta-node_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from delta_node.crypto.shamir import _native, field  # noqa: E402

dev = torch.device("cuda", 0)
for pre in (1, 333, 400, 560):
    for n in (1000, 40000):
        for pc in ("1", "0"):
            os.environ["DN_MT_PC_FORCE"] = pc
            a = random.Random(pre + n)
            a.getrandbits(32 * pre)
            b = random.Random()
            b.setstate(a.getstate())
            sec = torch.randint(-(1 << 62), 1 << 62, (n,), dtype=torch.int64, device=dev,
                                generator=torch.Generator(device=dev).manual_seed(n))
            got = torch.zeros((5, field.vec_bytes(n)), dtype=torch.uint8, device=dev)
            ok = _native.mt_split_device(a, sec, got, n, 3, 5)
            co = torch.from_numpy(_native.mt_draw_coeffs(b, n, 2)).to(dev)
            want = torch.zeros_like(got)
            _native.split_u64(sec, co, want, n, 3, 5)
            res = {"pre": pre, "n": n, "pc": pc, "ok": ok, "state": a.getstate() == b.getstate()}
            g, w = got.cpu().numpy(), want.cpu().numpy()
            for r in range(5):
                bad = np.nonzero((field.vec_to_limbs(g[r], n) != field.vec_to_limbs(w[r], n)).any(axis=1))[0]
                res[f"row{r}"] = [int(len(bad))] + [int(x) for x in bad[:6]]
            print(json.dumps(res), flush=True)
