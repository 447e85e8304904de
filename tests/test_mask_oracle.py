"""Pin the mask-PRG oracle (oracle/py_mask.py) and the host seeding of the
native library to the reference's make_mask outputs (tests/golden/mask.npz,
generated from delta_node/utils/arr.py) and to numpy itself.  CPU only."""
import hashlib
import os
import random

import numpy as np
import pytest

from delta_node.utils import _mask_native as mn
from golden.fixtures import HERE
from oracle import py_mask as pm

MAN = __import__("json").load(open(os.path.join(HERE, "mask_manifest.json")))
Z = np.load(os.path.join(HERE, "mask.npz"), allow_pickle=False)


def _seed(case):
    return bytes.fromhex(case["seed_hex"]) if "seed_hex" in case else case["seed_int"]


def test_py_oracle_matches_reference_masks():
    for case in MAN["cases"]:
        got = pm.make_mask(_seed(case), tuple(case["shape"]))
        assert np.array_equal(got, Z[case["key"]]), case["key"]


def test_numpy_is_the_reference_generator():
    for case in MAN["cases"]:
        assert np.array_equal(pm.make_mask_numpy(_seed(case), tuple(case["shape"])), Z[case["key"]])
    d = MAN["digests"][0]
    m = pm.make_mask_numpy(bytes.fromhex(d["seed_hex"]), (d["n"],))
    assert hashlib.sha256(m.tobytes()).hexdigest() == d["sha256"]


def test_native_host_seeding_matches_oracle_and_numpy():
    rng = random.Random(9)
    seeds = [bytes(rng.getrandbits(8) for _ in range(32)) for _ in range(20)] + [0, 1, 2**64 + 5, b""]
    for s in seeds:
        if s == b"":
            continue
        g = mn.pcg64(s)
        st, inc = pm.pcg64_init(s)
        assert (g.state, g.inc) == (st, inc)
        ref = np.random.PCG64(np.random.SeedSequence(s if isinstance(s, int) else list(s))).state["state"]
        assert (g.state, g.inc) == (ref["state"], ref["inc"])


def test_rejection_path_restated():
    seed = bytes(range(32))
    low, high = -3 * 2**61, 3 * 2**61  # threshold 2^62: a quarter of the draws are rejected
    out, rej = pm.bounded_int64(seed, 3000, low, high, return_raw=True)
    assert len(rej) > 500
    ref = np.random.default_rng(list(seed)).integers(low, high, size=3000, dtype=np.int64)
    assert np.array_equal(np.array(out, dtype=np.int64), ref)


def test_precision_fixture_is_numpy_semantics():
    with np.errstate(invalid="ignore", over="ignore"):
        assert np.array_equal(pm.fix_precision(Z["fix_in"], 8), Z["fix8"])
    assert np.array_equal(pm.unfix_precision(Z["unfix_in"], 8), Z["unfix8"])


def test_mask_exports():
    L = mn.lib()
    assert all(hasattr(L, s) for s in mn.EXPORTS)
