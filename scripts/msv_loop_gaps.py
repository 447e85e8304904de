#!/usr/bin/env python3
"""make_shares_vec (3-of-5, default pooled output) back to back: wall time per
call, and — under `rocprofv3 --kernel-trace --memory-copy-trace`, summarised
by `--summary DIR` — each call's GPU span and the idle gap before the next
call's first op (the host's share of a call in a loop).  The library is the
one DN_SHAMIR_LIB selects (A/B of variants).  One JSON line.
usage: msv_loop_gaps.py [log2n [default|caller|phases]] | msv_loop_gaps.py --summary DIR
caller: one pooled block allocated once and passed as out=; phases: the host
time of the pool allocation and free alone (no GPU work between)."""
import csv
import glob
import json
import os
import sys
import time

if len(sys.argv) > 2 and sys.argv[1] == "--summary":
    ops = []
    for f in glob.glob(f"{sys.argv[2]}/**/*kernel_trace.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            ops.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:40]))
    for f in glob.glob(f"{sys.argv[2]}/**/*memory_copy_trace.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            ops.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "copy"))
    ops.sort()
    # a call ends with its generation kernel; the next op starts the next call
    gens = [i for i, o in enumerate(ops) if "mt_gen" in o[2]]
    calls = []
    for a, b in zip(gens, gens[1:]):
        first = a + 1  # the next call's first op
        calls.append({"gap_us": (ops[first][0] - ops[a][1]) / 1e3,
                      "span_us": (ops[b][1] - ops[first][0]) / 1e3,
                      "gen_us": (ops[b][1] - ops[b][0]) / 1e3})
    print(json.dumps({"calls": calls[-8:]}))
    sys.exit(0)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "delta-node_amd"))

import torch  # noqa: E402

from delta_node.crypto import shamir  # noqa: E402

from delta_node.crypto.shamir import field, memory  # noqa: E402

lg = int(sys.argv[1]) if len(sys.argv) > 1 else 24
mode = sys.argv[2] if len(sys.argv) > 2 else "default"
N = 1 << lg
dev = torch.device("cuda", 0)
sec = torch.randint(-(1 << 62), 1 << 62, (N,), dtype=torch.int64, device=dev)
ss = shamir.SecretShare(3)
ss.random.seed(lg)
fixed = memory.share_block((5, field.vec_bytes(N)), dev) if mode == "caller" else None


def call():
    if mode == "phases":
        sh = memory.share_block((5, field.vec_bytes(N)), dev)
    else:
        sh = ss.make_shares_vec(sec, 5, out=fixed)
    del sh


for _ in range(3):
    call()
torch.cuda.synchronize()
walls = []
for _ in range(12):
    t0 = time.perf_counter()
    call()
    walls.append((time.perf_counter() - t0) * 1e3)
torch.cuda.synchronize()
walls.sort()
print(json.dumps({"lib": os.path.basename(os.environ.get("DN_SHAMIR_LIB", "libdn_shamir.so")), "log2n": lg,
                  "mode": mode, "ms_median": walls[len(walls) // 2], "ms_min": walls[0], "ms_max": walls[-1]}))
