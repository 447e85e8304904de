#!/usr/bin/env python3
"""Run selected bench.py rows alone (one JSON line): ROWS=byte_api,draw_split python scripts/rows_probe.py"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

import torch  # noqa: E402

dev = torch.device("cuda", 0)
out = {}
for r in os.environ.get("ROWS", "byte_api,draw_split").split(","):
    if r == "byte_api":
        out[r] = bench.byte_api_row()
    elif r == "rows":  # every row of bench.py's rows_bench (mask, codec, envelope, PRNG split, sum, MiMC7)
        out[r] = bench.rows_bench(dev, int(os.environ.get("LOG2N", "24")))
    elif r == "mask":
        out[r] = bench.mask_row(dev, int(os.environ.get("LOG2N", "24")))
    elif r == "draw_split":
        out[r] = bench.draw_split_row(dev, int(os.environ.get("LOG2N", "24")))
print(json.dumps(out))
