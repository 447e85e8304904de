#!/usr/bin/env python3
"""How the fused MT draw + split's generation time scales with the substreams
in flight (can half the substreams, started while the jump
level still runs, keep HBM busy?).  Tuning build, DN_MT_GEN_SUBS = K launches
only the first K of the 2^24 draw's 2048 substream workgroups (a timing probe:
partial output).  Run under `rocprofv3 --kernel-trace --stats` for per-kernel
times; prints the wall time per call for each K as JSON lines."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "delta-node_amd"))

import torch  # noqa: E402

from delta_node.crypto import shamir  # noqa: E402
from delta_node.crypto.shamir import _native, field  # noqa: E402

N = 1 << 24
dev = torch.device("cuda", 0)
sec = torch.randint(-(1 << 62), 1 << 62, (N,), dtype=torch.int64, device=dev)
out = torch.empty((5, field.vec_bytes(N)), dtype=torch.uint8, device=dev)
with _native.library(_native.TUNING_LIB):
    for k in (int(x) for x in os.environ.get("KS", "2049,1024,512,256").split(",")):
        os.environ["DN_MT_GEN_SUBS"] = str(k)
        ts = []
        for r in range(6):
            ss = shamir.SecretShare(3)
            ss.random.seed(r)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            try:
                ss.make_shares_vec(sec, 5, out=out)
            except Exception as e:  # the partial draw may leave a rejected-draw flag unset / state unchecked
                print(json.dumps({"K": k, "error": str(e)[:200]}), flush=True)
                break
            torch.cuda.synchronize()
            if r:
                ts.append((time.perf_counter() - t0) * 1e3)
        print(json.dumps({"K": k, "call_ms_best": min(ts) if ts else None, "call_ms": ts}), flush=True)
    os.environ.pop("DN_MT_GEN_SUBS", None)
