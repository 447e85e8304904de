#!/usr/bin/env python3
"""bench.py with memory.PROBE_TRIES_SMALL set to argv[1] (an A/B of the probe's
tries for share blocks under 1 GiB); the remaining arguments go to bench.py."""
import os
import runpy
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "delta-node_amd"))
from delta_node.crypto.shamir import memory  # noqa: E402

memory.PROBE_TRIES_SMALL = int(sys.argv[1])
sys.argv = [os.path.join(ROOT, "bench.py")] + sys.argv[2:]
runpy.run_path(sys.argv[0], run_name="__main__")
