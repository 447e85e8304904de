#!/usr/bin/env python3
"""Golden fixtures for the mask-PRG row from the REAL reference (build container only).

Loads /root/reference/delta_node/utils/arr.py by file path (it imports only
numpy and the stdlib) and records `make_mask(seed, shape)` outputs for bytes
and int seeds, plus SHA-256 digests of large masks.  precision.py cannot be
imported (it imports the absent `delta` package, precision.py:2); its two
numpy expressions (precision.py:5-15) are evaluated here on numpy directly to
record fix/unfix expectations, including NaN / inf / out-of-range inputs.

Outputs: tests/golden/mask.npz, tests/golden/mask_manifest.json.
"""
import hashlib
import importlib.util
import json
import os
import random

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
spec = importlib.util.spec_from_file_location("ref_arr", "/root/reference/delta_node/utils/arr.py")
ref_arr = importlib.util.module_from_spec(spec)
spec.loader.exec_module(ref_arr)


def main():
    rng = random.Random(47)
    seeds = [bytes(rng.getrandbits(8) for _ in range(32)) for _ in range(6)] + [b"\x00" * 32, b"\xff" * 32, b"\x01"]
    int_seeds = [0, 1, 12345, 2 ** 40 + 7]
    shapes = [(10,), (3, 7), (1000,), (64, 17)]
    arrays = {}
    cases = []
    for i, s in enumerate(seeds):
        for j, shp in enumerate(shapes):
            key = f"b{i}_{j}"
            arrays[key] = ref_arr.make_mask(s, shp)
            cases.append({"key": key, "seed_hex": s.hex(), "shape": list(shp)})
    for i, s in enumerate(int_seeds):
        key = f"i{i}"
        arrays[key] = ref_arr.make_mask(s, (500,))
        cases.append({"key": key, "seed_int": s, "shape": [500]})
    digests = []
    for i, (s, n) in enumerate([(seeds[0], 1 << 16), (seeds[1], 1 << 20), (seeds[2], 1 << 24)]):
        m = ref_arr.make_mask(s, (n,))
        digests.append({"seed_hex": s.hex(), "n": n, "sha256": hashlib.sha256(m.tobytes()).hexdigest()})
    # precision.py:5-15 expressions, evaluated on numpy
    fx_in = np.concatenate([np.random.default_rng(5).standard_normal(200) * 1e3,
                            np.array([0.0, -0.0, 1e-9, -1e-9, 0.5, -0.5, 123456.789, 9.2e10, -9.2e10, 9.3e10,
                                      np.nan, np.inf, -np.inf, 1e300, -1e300])])
    with np.errstate(invalid="ignore", over="ignore"):
        fixed8 = (fx_in.astype(np.float64) * (10 ** 8)).astype(np.int64)
    ints = np.random.default_rng(6).integers(-(1 << 62), 1 << 62, 300, dtype=np.int64)
    unfixed8 = ints.astype(np.float64) / (10 ** 8)
    arrays.update({"fix_in": fx_in, "fix8": fixed8, "unfix_in": ints, "unfix8": unfixed8})
    np.savez_compressed(os.path.join(HERE, "mask.npz"), **arrays)
    man = {"generator": "tests/golden/make_golden_mask.py (reference delta_node/utils/arr.py loaded by path)",
           "numpy": np.__version__, "cases": cases, "digests": digests}
    json.dump(man, open(os.path.join(HERE, "mask_manifest.json"), "w"), indent=1)
    print("wrote", len(cases), "cases,", len(digests), "digests")


if __name__ == "__main__":
    main()
