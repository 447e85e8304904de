#!/usr/bin/env python3
"""Debug: coefficient draw (T = 0) and fused split for substream 0 inside the
caller's array, two-wave vs one-wave kernel (tuning library, DN_MT_PC_FORCE),
against the host draw: first differing tile / element per row."""
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
for pre in (1, 333, 560):
    for n in (1000, 40000):
        for pc in ("1", "0"):
            os.environ["DN_MT_PC_FORCE"] = pc
            a = random.Random(pre + n)
            a.getrandbits(32 * pre)
            b = random.Random()
            b.setstate(a.getstate())
            got = torch.zeros((2, field.vec_bytes(n)), dtype=torch.uint8, device=dev)
            ok = _native.mt_draw_coeffs_device(a, n, 2, got)
            want = _native.mt_draw_coeffs(b, n, 2)
            g = got.cpu().numpy()
            res = {"pre": pre, "n": n, "pc": pc, "ok": ok, "state": a.getstate() == b.getstate()}
            for r in range(2):
                gl = field.vec_to_limbs(g[r], n)
                wl = field.vec_to_limbs(want[r], n)
                bad = np.nonzero((gl != wl).any(axis=1))[0]
                res[f"row{r}_bad"] = [int(len(bad))] + [int(x) for x in bad[:8]]
            print(json.dumps(res), flush=True)
