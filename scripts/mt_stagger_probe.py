#!/usr/bin/env python3
"""Do the fused generation kernel's waves stay in step (all generating, then
all emitting)?  mt_gen_kernel<3> at 2^24 on a share block with the tuning
build's DN_MT_STAGGER = k: substream s sleeps (s % 4) * k * ~3.4 us before
its first group, so a quarter of the waves start each phase offset.  Run under
rocprofv3 --kernel-trace with DN_SHAMIR_LIB = the tuning library; REPS calls
per setting in the printed order (scripts/mt_gen_probe_summary.py)."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "delta-node_amd"))

import torch  # noqa: E402

from delta_node.crypto import shamir  # noqa: E402
from delta_node.crypto.shamir import _native, field, memory  # noqa: E402

assert "tuning" in _native.lib_path(), "run with DN_SHAMIR_LIB=.../libdn_shamir_tuning.so"
N = 1 << 24
REPS = int(os.environ.get("REPS", "5"))
dev = torch.device("cuda", 0)
sec = torch.randint(-(1 << 62), 1 << 62, (N,), dtype=torch.int64, device=dev)
blk = memory.share_block((5, field.vec_bytes(N)), dev)
ss = shamir.SecretShare(3)
ss.random.seed(5)
order = []
for st in ("0", "1", "2", "4", "0", "1"):
    os.environ["DN_MT_STAGGER"] = st
    for _ in range(REPS):
        ss.make_shares_vec(sec, 5, out=blk)
        torch.cuda.synchronize()
        time.sleep(0.001)
    order.append({"block": 0, "kind": "share_block", "back": 1, "probe": 0, "stagger": int(st), "calls": REPS})
print(json.dumps({"order": order}))
