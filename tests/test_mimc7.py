"""MiMC7 commitments.

CPU: the oracle (oracle/py_mimc7.py) against the reference's own
known-answer tests (tests/mimc7_test.py:5-97 values, tests/golden/mimc7_kat.json).
GPU: the HIP kernels against the same KATs and against the oracle on random
data (bit-exact field arithmetic).
"""
import json
import os
import random

import numpy as np
import pytest

from golden.fixtures import HERE
from oracle import py_mimc7 as om

KAT = json.load(open(os.path.join(HERE, "mimc7_kat.json")))


def kat_data():
    return np.hstack([np.array(KAT["data_x"], dtype=np.float64), np.array(KAT["data_y"], dtype=np.uint8)[:, None]])


def hex32(b: bytes) -> str:
    return "0x" + b.hex().rjust(64, "0")


def test_oracle_matches_reference_kats():
    assert str(om.mimc7_hash(1, 0)) == KAT["hash_1_0"]
    assert hex32(om.weight_commitment(KAT["weight"])) == KAT["weight_commitment"]
    res = om.data_commitment(kat_data())
    assert len(res) == 1 and hex32(res[0]) == KAT["data_commitment"]


@pytest.mark.gpu
def test_gpu_matches_reference_kats():
    from delta_node.utils import mimc7

    assert mimc7.mimc7_hash([1], [0]) == [int(KAT["hash_1_0"])]
    assert hex32(mimc7.calc_weight_commitment(KAT["weight"])) == KAT["weight_commitment"]
    res = mimc7.calc_data_commitment(kat_data())
    assert len(res) == 1 and hex32(res[0]) == KAT["data_commitment"]


@pytest.mark.gpu
def test_gpu_vs_oracle_random():
    from delta_node.utils import mimc7

    rng = random.Random(1)
    xs = [rng.randrange(om.Q) for _ in range(300)] + [0, 1, om.Q - 1]
    ks = [rng.randrange(om.Q) for _ in range(300)] + [om.Q - 1, 0, om.Q - 1]
    assert mimc7.mimc7_hash(xs, ks) == [om.mimc7_hash(x, k) for x, k in zip(xs, ks)]
    w = np.random.default_rng(2).standard_normal(257) * np.array([1, 1e5, 1e-7] * 85 + [1, 1])
    w[:4] = [0.0, -0.0, 1e30, -1e30]
    assert mimc7.calc_weight_commitment(w) == om.weight_commitment(w)
    data = np.random.default_rng(3).standard_normal((300, 5)) * 10
    data[:, -1] = np.random.default_rng(4).integers(0, 2, 300)
    data[5, 2] = -3.3e20
    assert mimc7.calc_data_commitment(data) == om.data_commitment(data)
