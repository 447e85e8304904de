"""MiMC7 commitments.

CPU: the oracle (oracle/py_mimc7.py) against the reference's own
known-answer tests (tests/mimc7_test.py:5-97 values, tests/golden/mimc7_kat.json);
calc_weight_commitment's native host chain (dn_mimc7_weight_commitment_host)
against the same KAT and the oracle, including weights far beyond 2^253 / 10^8,
signed zeros, subnormals and the int() errors; utils.constant against the
oracle's q / cts.
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


def test_host_weight_commitment_matches_reference_kat():
    from delta_node.utils import calc_weight_commitment

    assert hex32(calc_weight_commitment(KAT["weight"])) == KAT["weight_commitment"]
    assert calc_weight_commitment([]) == om.weight_commitment([])


def test_host_weight_commitment_vs_oracle_extremes():
    from delta_node.utils import calc_weight_commitment

    rng = np.random.default_rng(5)
    w = rng.standard_normal(400) * np.array([1, 1e5, 1e-7, 1e30] * 100)
    w[:16] = [0.0, -0.0, 5e-324, -5e-324, 1e-8, -1e-8, 1.5e-8, 1.7976931348623157e300, -1.7976931348623157e300,
              1.4474011154664524e245, -1.4474011154664524e245, 1.0944121435919637e245, 2.0e244, 9.9e-9, 2 ** 200,
              -(2 ** 203)]
    # around q/2 and q (divided by 10^8): both sides of the min(a, q - a) branch
    for v in (om.Q // 2, om.Q // 2 + 1, om.Q - 1, om.Q, om.Q + 1, 2 ** 256):
        w = np.append(w, [v / 1e8, -v / 1e8, np.nextafter(v / 1e8, 0), np.nextafter(v / 1e8, np.inf)])
    assert calc_weight_commitment(w) == om.weight_commitment(w)
    for x in w:  # one weight at a time: each conversion on its own
        assert calc_weight_commitment([x]) == om.weight_commitment([x]), x
    # float32 input converts to float64 first (numpy 1.22 casting of float32 * 10**8)
    w32 = rng.standard_normal(50).astype(np.float32)
    assert calc_weight_commitment(w32) == om.weight_commitment([np.float64(x) for x in w32])


def test_host_weight_commitment_errors_as_int():
    from delta_node.utils import calc_weight_commitment

    with pytest.raises(ValueError):
        calc_weight_commitment([1.0, float("nan")])
    with pytest.raises(OverflowError):
        calc_weight_commitment([float("inf")])
    with pytest.raises(OverflowError):
        calc_weight_commitment([1e301])  # 1e301 * 10^8 overflows the float multiply, as in the reference


def test_constant_matches_reference_values():
    from delta_node.utils import constant

    assert constant.q() == om.Q
    assert constant.cts() == list(om.CTS) and len(constant.cts()) == 13
    assert constant.data_block_size() == 128


def test_constant_literals_equal_library_params():
    """utils/constant.py holds plain literals (importable without the native
    library, as the reference's); the kernels' copy must be the same."""
    import ctypes

    from delta_node.crypto.shamir import _native
    from delta_node.utils import constant

    L = _native.lib()
    qb = (ctypes.c_uint32 * 8)()
    cb = (ctypes.c_uint32 * (13 * 8))()
    L.dn_mimc7_params.restype = ctypes.c_int
    L.dn_mimc7_params.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    assert L.dn_mimc7_params(ctypes.addressof(qb), ctypes.addressof(cb)) == 0
    assert int.from_bytes(bytes(qb), "little") == constant.q()
    raw = bytes(cb)
    assert [int.from_bytes(raw[32 * i:32 * (i + 1)], "little") for i in range(13)] == constant.cts()


def test_calc_commitment_and_npz_helpers(tmp_path):
    import hashlib
    import io

    from delta_node.utils import calc_commitment, dump_arr, load_arr

    assert calc_commitment(b"abc") == hashlib.sha256(b"abc").digest()
    assert calc_commitment(io.BytesIO(b"line1\nline2\n")) == hashlib.sha256(b"line1\nline2\n").digest()
    assert calc_commitment([b"ab", b"c"]) == hashlib.sha256(b"abc").digest()
    arr = np.arange(12, dtype=np.int64).reshape(3, 4)
    buf = io.BytesIO()
    dump_arr(buf, arr)
    buf.seek(0)
    np.testing.assert_array_equal(load_arr(buf), arr)
    f = tmp_path / "plain.npy"
    np.save(f, arr.astype(np.float32))
    with open(f, "rb") as fh:
        got = load_arr(fh)
    assert got.dtype == np.float32 and np.array_equal(got, arr)


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
    assert mimc7.weight_commitment_device(w) == om.weight_commitment(w)
    assert hex32(mimc7.weight_commitment_device(KAT["weight"])) == KAT["weight_commitment"]
    data = np.random.default_rng(3).standard_normal((300, 5)) * 10
    data[:, -1] = np.random.default_rng(4).integers(0, 2, 300)
    data[5, 2] = -3.3e20
    assert mimc7.calc_data_commitment(data) == om.data_commitment(data)


@pytest.mark.gpu
@pytest.mark.parametrize("blocks", [2048 + 3, 8192 + 5])
def test_gpu_packed_merkle_blocks_equal_single_blocks(blocks):
    """Many blocks take the packed Merkle kernel (4 or 16 blocks per
    workgroup, levels packed onto full waves, a partial last workgroup): each
    root equals the commitment of its 128 rows alone (one block, the
    one-block-per-workgroup kernel the oracle pins), for blocks at the start,
    around workgroup boundaries and at the end."""
    import torch

    from delta_node.utils import mimc7

    rows = blocks * 128 - 77  # the last block is zero-padded
    rng = np.random.default_rng(blocks)
    data = rng.standard_normal((rows, 6))
    data[:, -1] = rng.integers(0, 2, rows)
    dev = torch.device("cuda", 0)
    roots = mimc7.calc_data_commitment(torch.from_numpy(data).to(dev))
    assert len(roots) == blocks
    for b in sorted({0, 1, 3, 4, 15, 16, 17, blocks // 2, blocks - 6, blocks - 2, blocks - 1}):
        one = mimc7.calc_data_commitment(torch.from_numpy(data[128 * b:128 * (b + 1)]).to(dev))
        assert roots[b] == one[0], b
