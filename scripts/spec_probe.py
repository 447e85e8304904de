#!/usr/bin/env python3
"""What a speculative next-call jump level could save in a make_shares_vec
loop (its second variant).  Tuning build,
DN_MT_SPEC_PROBE (timing probe only: the output is wrong):
  0  the product sequence (jump levels, then the generation)
  1  the jump levels skipped: the generation alone per call (the floor)
  2  skipped, the same levels on a side stream into a buffer of their own,
     launched before the generation and awaited by the next call's generation
  3  as 2, launched after the generation
Back-to-back 2^24 3-of-5 calls into one share block; wall ms per call (median
of 30 after 5 warm-up), modes alternated over ROUNDS rounds.  JSON lines."""
import json
import os
import statistics
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
modes = [int(m) for m in os.environ.get("MODES", "0,1,2,3").split(",")]
with _native.library(_native.TUNING_LIB):
    ss = shamir.SecretShare(3)
    ss.random.seed(1)
    ss.make_shares_vec(sec, 5, out=out)  # windows in the scratch
    for rnd in range(int(os.environ.get("ROUNDS", "2"))):
        for m in modes:
            os.environ["DN_MT_SPEC_PROBE"] = str(m)
            ts, err = [], None
            for i in range(35):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                try:
                    ss.make_shares_vec(sec, 5, out=out)
                except Exception as e:  # stale windows: a flagged draw is possible, if unlikely
                    err = str(e)[:200]
                    ss.random.seed(i)
                    continue
                torch.cuda.synchronize()
                if i >= 5:
                    ts.append((time.perf_counter() - t0) * 1e3)
            print(json.dumps({"round": rnd, "mode": m, "ms_median": statistics.median(ts) if ts else None,
                              "ms_min": min(ts) if ts else None, "n": len(ts), "error": err}), flush=True)
    os.environ.pop("DN_MT_SPEC_PROBE", None)
    torch.cuda.synchronize()
