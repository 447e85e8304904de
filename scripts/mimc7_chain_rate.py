#!/usr/bin/env python3
"""MiMC7 weight commitment (utils/mimc7.py:58-60): the host chain
(calc_weight_commitment, dn_mimc7_weight_commitment_host), the same chain on
one device lane (weight_commitment_device) and the pure-Python restatement
(oracle/py_mimc7.py) on the same weights.  One JSON line."""
import os, sys, time, json
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "delta-node_amd"), ROOT]
import numpy as np, torch
from delta_node.utils import mimc7
from oracle import py_mimc7
w = np.random.default_rng(0).standard_normal(200000) * 0.1
wdev = torch.from_numpy(w[:4000]).cuda()
mimc7.weight_commitment_device(wdev[:10]); torch.cuda.synchronize()
out = {}
for n in (2000, 200000):
    t0 = time.perf_counter(); mimc7.calc_weight_commitment(w[:n]); out[f"host_{n}_s"] = time.perf_counter() - t0
t0 = time.perf_counter(); d = mimc7.weight_commitment_device(wdev[:2000]); out["device_2000_s"] = time.perf_counter() - t0
t0 = time.perf_counter(); c = py_mimc7.weight_commitment(w[:2000]); out["py_2000_s"] = time.perf_counter() - t0
out["equal_2000"] = c == mimc7.calc_weight_commitment(w[:2000]) == d
print(json.dumps(out))
