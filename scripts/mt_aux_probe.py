#!/usr/bin/env python3
"""Same-process A/B of the fused draw + split's share-store cache policy
(DN_MT_STORE_AUX, tuning library): make_shares_vec(2^24 int64, 5) on
SecretShare(3), the same output buffer for every variant, rounds
interleaved.  OUTS=chunk: the outputs are memory.share_block blocks (2 MiB
physical chunks).  PROBE=1: also time DN_MT_PROBE=1 (generation only) and 2
(emission only) with the default policy.  Prints one JSON line."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "delta-node_amd"))
os.environ["DN_SHAMIR_LIB"] = os.path.join(ROOT, "delta-node_amd", "lib", "libdn_shamir_tuning.so")

import torch  # noqa: E402

from delta_node.crypto import shamir  # noqa: E402
from delta_node.crypto.shamir import field, memory  # noqa: E402

N = 1 << 24
dev = torch.device("cuda", 0)
sec = torch.randint(-(1 << 62), 1 << 62, (N,), dtype=torch.int64, device=dev)
if os.environ.get("OUTS") == "chunk":
    outs = [memory.chunked_block((5, field.vec_bytes(N)), device=dev) for _ in range(2)]
else:
    outs = [torch.empty((5, field.vec_bytes(N)), dtype=torch.uint8, device=dev) for _ in range(2)]
auxes = os.environ.get("AUXES", "2,0,1,16,18").split(",")
res = {f"buf{b}": {a: [] for a in auxes} for b in range(len(outs))}
ref = None
for rnd in range(3):
    for b, out in enumerate(outs):
        for a in auxes:
            os.environ["DN_MT_STORE_AUX"] = a
            ss = shamir.SecretShare(3)
            ss.random.seed(9)
            ss.make_shares_vec(sec, 5, out=out)
            torch.cuda.synchronize()
            if ref is None:
                ref = out.clone()
            assert torch.equal(out, ref), a
            t0 = time.perf_counter()
            for _ in range(5):
                ss.make_shares_vec(sec, 5, out=out)
            torch.cuda.synchronize()
            res[f"buf{b}"][a].append((time.perf_counter() - t0) / 5 * 1e3)
probe = {}
if os.environ.get("PROBE") == "1":
    os.environ.pop("DN_MT_STORE_AUX", None)
    for pr in ("1", "2", "0"):
        os.environ["DN_MT_PROBE"] = pr
        for b, out in enumerate(outs):
            ss = shamir.SecretShare(3)
            ss.random.seed(9)
            ss.make_shares_vec(sec, 5, out=out)
            torch.cuda.synchronize()
            ms = []
            for _ in range(3):
                t0 = time.perf_counter()
                for _ in range(5):
                    ss.make_shares_vec(sec, 5, out=out)
                torch.cuda.synchronize()
                ms.append((time.perf_counter() - t0) / 5 * 1e3)
            probe[f"probe{pr}_buf{b}"] = min(ms)
    os.environ.pop("DN_MT_PROBE", None)
print(json.dumps({"outs": os.environ.get("OUTS", "torch"), "probe_ms": probe,
                  "make_shares_vec_ms_2e24_by_store_aux": {k: {a: min(v) for a, v in d.items()} for k, d in res.items()},
                  "all": res}))
