#!/usr/bin/env python3
"""The 2^24 direct jump level by mt_jump_kernel<16> (83 KB table, b64
reads, one workgroup per CU) vs mt_jumpc_kernel<16, 4> (45 KB contiguous
table, b32 reads, two workgroups per CU), tuning build: lone
make_shares_vec(2^24) calls (fresh SecretShare each, no speculation) into a
share block, wall ms per call (best of 8) per configuration (DN_MT_JUMP4B,
DN_MT_PARTS_B), alternated over ROUNDS rounds.  Run under rocprofv3
--kernel-trace for the jump kernels' own durations.  JSON lines."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "delta-node_amd"))

import torch  # noqa: E402

from delta_node.crypto import shamir  # noqa: E402
from delta_node.crypto.shamir import _native, field, memory  # noqa: E402

N = 1 << 24
dev = torch.device("cuda", 0)
torch.cuda.set_device(0)
sec = torch.randint(-(1 << 62), 1 << 62, (N,), dtype=torch.int64, device=dev)
out = memory.share_block((5, field.vec_bytes(N)), dev)
os.environ["DN_MT_SPEC"] = "0"
configs = [("0", None), ("1", "8"), ("1", "4")]
with _native.library(_native.TUNING_LIB):
    for rnd in range(int(os.environ.get("ROUNDS", "2"))):
        for j4, pb in configs:
            os.environ["DN_MT_JUMP4B"] = j4
            if pb:
                os.environ["DN_MT_PARTS_B"] = pb
            else:
                os.environ.pop("DN_MT_PARTS_B", None)
            ts = []
            for r in range(9):
                ss = shamir.SecretShare(3)
                ss.random.seed(100 * rnd + r)
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                ss.make_shares_vec(sec, 5, out=out)
                torch.cuda.synchronize()
                if r:
                    ts.append((time.perf_counter() - t0) * 1e3)
            print(json.dumps({"round": rnd, "jump4b": j4, "parts": pb or "default", "ms_best": min(ts),
                              "ms_median": sorted(ts)[len(ts) // 2]}), flush=True)
