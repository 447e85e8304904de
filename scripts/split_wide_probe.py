#!/usr/bin/env python3
"""A/B of the split's store width (tuning library): one element per lane
(split_kernel, 4-B plane accesses) vs E = 2 / 4 consecutive elements per lane
(split_wide_kernel, 8-B / 16-B accesses), each over several grid caps, on
several share-buffer allocations in one process; beside each, the same-buffer
ceiling dn_diag_tile_stream (the split's bytes with 16-B accesses and no
arithmetic).  Parity: every variant's shares equal the one-element split's.

    DN_SHAMIR_LIB=delta-node_amd/lib/libdn_shamir_tuning.so python scripts/split_wide_probe.py
"""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("DN_SHAMIR_LIB", os.path.join(ROOT, "delta-node_amd", "lib", "libdn_shamir_tuning.so"))
sys.path.insert(0, os.path.join(ROOT, "delta-node_amd"))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from delta_node.crypto import shamir  # noqa: E402
from delta_node.crypto.shamir import _native, field  # noqa: E402

LOG2N = int(os.environ.get("PROBE_LOG2N", "24"))
ALLOCS = int(os.environ.get("PROBE_ALLOCS", "3"))
REPS = 5
N = 1 << LOG2N
VB = field.vec_bytes(N)
dev = torch.device("cuda", 0)
diag = ctypes.CDLL(os.path.join(ROOT, "delta-node_amd", "lib", "libdn_diag.so"))
vp = ctypes.c_void_p


def ceiling(sec, coeffs, shares, t, n, grid):
    ins = (vp * 8)(sec.data_ptr(), *[coeffs[j].data_ptr() for j in range(t - 1)])
    ibpt = (ctypes.c_uint32 * 8)(2048, *([field.TILE_BYTES] * (t - 1)))
    outs = (vp * 16)(*[shares[x].data_ptr() for x in range(n)])
    obpt = (ctypes.c_uint32 * 16)(*([field.TILE_BYTES] * n))
    rc = diag.dn_diag_tile_stream(ins, ibpt, t, outs, obpt, n, ctypes.c_uint64(N // 256), grid,
                                  vp(torch.cuda.current_stream().cuda_stream))
    assert rc == 0, rc


def timed(fn):
    fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(REPS):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / REPS


def run(t, n, variants, grids):
    rng = np.random.default_rng(1)
    sec = torch.from_numpy(rng.integers(-(1 << 63), (1 << 63) - 1, size=N, endpoint=True, dtype=np.int64)).to(dev)
    ss = shamir.SecretShare(t)
    ss.random.seed(1)
    coeffs = ss.draw_coeffs_vec(N, dev)
    per_elem = 8 + (t - 1) * 66 + n * 66
    ref = None
    for a in range(ALLOCS):
        shares = torch.empty((n, VB), dtype=torch.uint8, device=dev)
        for rnd in range(2):
            for E, cap in variants:
                os.environ["DN_SPLIT_E"] = str(E)
                if cap:
                    os.environ["DN_GRID_CAP"] = str(cap)
                else:
                    os.environ.pop("DN_GRID_CAP", None)
                ms = timed(lambda: _native.split_u64(sec, coeffs, shares, N, t, n))
                eq = None
                if rnd == 0:
                    dig = shares.view(torch.int64).sum(dim=1).cpu()
                    if ref is None and E == 0:
                        ref = (shares[:, :1 << 20].clone(), dig)
                    eq = bool(torch.equal(dig, ref[1]) and torch.equal(shares[:, :1 << 20], ref[0]))
                print(json.dumps({"t": t, "n": n, "alloc": a, "round": rnd, "E": E, "grid_cap": cap, "ms": ms,
                                  "GBps": N * per_elem / (ms * 1e-3) / 1e9, "equal_narrow": eq}), flush=True)
            os.environ.pop("DN_GRID_CAP", None)
            os.environ.pop("DN_SPLIT_E", None)
            for g in grids:
                ms = timed(lambda: ceiling(sec, coeffs, shares, t, n, g))
                print(json.dumps({"t": t, "n": n, "alloc": a, "round": rnd, "ceiling_grid": g, "ms": ms,
                                  "GBps": N * per_elem / (ms * 1e-3) / 1e9}), flush=True)
        del shares
        torch.cuda.empty_cache()


CASES = os.environ.get("PROBE_CASES", "t3,t5")
if "t3" in CASES:
    run(3, 5, [(0, 0), (0, 16384), (2, 0), (2, 1024), (2, 16384), (4, 0), (4, 512), (4, 2048), (4, 16384)],
        [256, 1024, 4096, 16384])
if "t5" in CASES:
    run(5, 9, [(0, 0), (2, 0), (2, 512), (2, 16384)], [256, 1024, 4096])
