#!/usr/bin/env python3
"""Anatomy of the fused MT draw + split's generation kernel on share blocks
(run under rocprofv3 --kernel-trace with DN_SHAMIR_LIB = the tuning library,
whose DN_MT_PROBE skips parts of mt_gen_kernel):
  probe 0  the full kernel;
  probe 1  generation only (no emission: temper, split, share stores);
  probe 2  emission only (from a stale ring; no MT appends);
each with DN_MT_BACK = 1 (the default: odd substreams forward, even ones
backward), 0 (every substream forward) and 2 (every inner one backward).
REPS calls per (block, probe), in the order printed; scripts/mt_gen_probe_summary.py
maps the trace's mt_gen_kernel<3, ...> launches back to them."""
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
vb = field.vec_bytes(N)
sec = torch.randint(-(1 << 62), 1 << 62, (N,), dtype=torch.int64, device=dev)
blocks = [("share_block", memory.share_block((5, vb), dev)),
          ("torch.empty", torch.empty((5, vb), dtype=torch.uint8, device=dev))]
ss = shamir.SecretShare(3)
ss.random.seed(5)
order = []
BACKS = os.environ.get("BACKS", "1,0,2").split(",")
PCS = os.environ.get("PCS", "").split(",") if os.environ.get("PCS") else [None]
for bi, (kind, blk) in enumerate(blocks):
  for pc in PCS:
    if pc is not None:
        os.environ["DN_MT_PC_FORCE"] = pc
    for back in BACKS:
        os.environ["DN_MT_BACK"] = back
        for probe in ("0", "1", "2"):
            os.environ["DN_MT_PROBE"] = probe
            for _ in range(REPS):
                ss.make_shares_vec(sec, 5, out=blk)
                torch.cuda.synchronize()
                time.sleep(0.001)
            order.append({"block": bi, "kind": kind, "back": int(back), "probe": int(probe), "calls": REPS,
                          "pc": pc})
os.environ.pop("DN_MT_PROBE")
os.environ.pop("DN_MT_BACK")
os.environ.pop("DN_MT_PC_FORCE", None)
if os.environ.get("NO_FG"):
    print(json.dumps({"order": order}))
    sys.exit(0)
# the pair boundary (mt_sub_range): forward groups per pair of 2 x 128 at t = 3;
# every split must give the same shares and the same final state
blk = blocks[0][1]
r0 = __import__("random").Random(77)
ss.random = r0
ss.make_shares_vec(sec, 5, out=blk)
order.append({"block": 0, "kind": "ref", "back": 1, "probe": 0, "calls": 1})
ref, ref_state = blk.clone(), ss.random.getstate()
same = {}
for fg in ("128", "120", "112", "104", "96", "136"):
    os.environ["DN_MT_FWD_GROUPS"] = fg
    for _ in range(REPS):
        ss.random = __import__("random").Random(77)
        ss.make_shares_vec(sec, 5, out=blk)
        torch.cuda.synchronize()
        time.sleep(0.001)
    same[fg] = bool(torch.equal(blk, ref)) and ss.random.getstate() == ref_state
    order.append({"block": 0, "kind": "share_block", "back": 1, "probe": 0, "fwd_groups": int(fg), "calls": REPS})
os.environ.pop("DN_MT_FWD_GROUPS")
print(json.dumps({"order": order, "fwd_groups_equal_output": same}))
