#!/usr/bin/env python3
"""MiMC7 weight commitment (utils/mimc7.py:58-60): the GPU's single sequential
chain (chain_kernel, one lane) vs the pure-Python restatement (oracle/py_mimc7.py)
on the same weights.  One JSON line."""
import os, sys, time, json
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "delta-node_amd"), ROOT]
import numpy as np, torch
from delta_node.utils import mimc7
from oracle import py_mimc7
w = np.random.default_rng(0).standard_normal(20000) * 0.1
mimc7.calc_weight_commitment(w[:10]); torch.cuda.synchronize()
out = {}
for n in (2000, 20000):
    t0 = time.perf_counter(); g = mimc7.calc_weight_commitment(w[:n]); gt = time.perf_counter() - t0
    out[f"gpu_{n}_s"] = gt
t0 = time.perf_counter(); c = py_mimc7.weight_commitment(w[:2000]); ct = time.perf_counter() - t0
out["py_2000_s"] = ct
out["equal_2000"] = c == mimc7.calc_weight_commitment(w[:2000])
print(json.dumps(out))
