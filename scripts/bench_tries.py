#!/usr/bin/env python3
"""bench.py with the share-block probe's tries set from argv[1] (an A/B of the
probe policy, memory.py): "SMALL" or "SMALL,LARGE,BUDGET_GIB[,FIRST_SMALL]"
sets PROBE_TRIES_SMALL (blocks under 1 GiB), PROBE_TRIES (1 GiB and up),
PROBE_BUDGET and PROBE_FIRST_SMALL; the remaining arguments go to bench.py."""
import os
import runpy
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "delta-node_amd"))
from delta_node.crypto.shamir import memory  # noqa: E402

vals = [int(v) for v in sys.argv[1].split(",")]
memory.PROBE_TRIES_SMALL = vals[0]
if len(vals) > 1:
    memory.PROBE_TRIES = vals[1]
    memory.PROBE_BUDGET = vals[2] << 30
if len(vals) > 3:
    memory.PROBE_FIRST_SMALL = vals[3]
sys.argv = [os.path.join(ROOT, "bench.py")] + sys.argv[2:]
runpy.run_path(sys.argv[0], run_name="__main__")
