#!/usr/bin/env python3
"""A/B of the MT19937 jump-table layouts (DN_MT_JUMP_LAYOUT, tuning build):
0 = 8-B pair planes (82 KB, one workgroup per CU), 1 = compact rows (44 KB,
three per CU).  Alternates the layouts in one process over the device draw of
2^24 x 2 coefficients (jump levels + generation); checks both against the
host draw.  Prints one JSON line per repetition."""
import json
import os
import random
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["DN_SHAMIR_LIB"] = os.path.join(ROOT, "delta-node_amd", "lib", "libdn_shamir_tuning.so")
sys.path.insert(0, os.path.join(ROOT, "delta-node_amd"))

import torch  # noqa: E402

from delta_node.crypto.shamir import _native, field  # noqa: E402

N, TM1 = 1 << int(os.environ.get("LOG2N", "24")), 2
dev = torch.device("cuda", 0)
blk = torch.empty((TM1, field.vec_bytes(N)), dtype=torch.uint8, device=dev)
want = torch.from_numpy(_native.mt_draw_coeffs(random.Random(11), N, TM1)).to(dev)
for rep in range(int(os.environ.get("REPS", "6"))):
    out = {"rep": rep}
    for lay in ("0", "1"):
        os.environ["DN_MT_JUMP_LAYOUT"] = lay
        b = random.Random(11)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        ok = _native.mt_draw_coeffs_device(b, N, TM1, blk)
        torch.cuda.synchronize()
        out[f"layout{lay}_draw_ms"] = (time.perf_counter() - t0) * 1e3
        out[f"layout{lay}_equal"] = bool(ok and torch.equal(blk, want))
    print(json.dumps(out), flush=True)
