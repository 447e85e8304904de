"""HIP mask PRG vs the reference's make_mask and numpy.

Checkers: tests/golden/mask.npz (outputs of the reference's
delta_node/utils/arr.py, incl. a 2^24-element digest) and numpy's own
Generator — numpy is the reference's PRG dependency and is present on the
GPU box, so full-size parity is checked against it directly.  Bit-exact.
"""
import hashlib
import os

import numpy as np
import pytest
import torch

from delta_node import utils
from delta_node.utils import _mask_native as mn
from delta_node.utils.mask import bounded_sum
from golden.fixtures import HERE
from oracle import py_mask as pm

pytestmark = pytest.mark.gpu
MAN = __import__("json").load(open(os.path.join(HERE, "mask_manifest.json")))
Z = np.load(os.path.join(HERE, "mask.npz"), allow_pickle=False)


def _seed(case):
    return bytes.fromhex(case["seed_hex"]) if "seed_hex" in case else case["seed_int"]


def test_make_mask_matches_reference_fixture():
    for case in MAN["cases"]:
        got = utils.make_mask(_seed(case), tuple(case["shape"]))
        assert got.dtype == np.int64 and got.shape == tuple(case["shape"])
        assert np.array_equal(got, Z[case["key"]]), case["key"]


def test_make_mask_digests_up_to_2e24():
    for d in MAN["digests"]:
        m = utils.make_mask(bytes.fromhex(d["seed_hex"]), (d["n"],))
        assert hashlib.sha256(m.tobytes()).hexdigest() == d["sha256"], d["n"]


@pytest.mark.parametrize("n", [1, 63, 64, 1000, 4095, 4097, 70001])
def test_make_mask_ragged_vs_numpy(n):
    seed = os.urandom(32)
    assert np.array_equal(utils.make_mask(seed, (n,)), pm.make_mask_numpy(seed, (n,)))


@pytest.mark.parametrize("k", [12, 16, 19])
def test_masked_sum_matches_reference_composition(k):
    """runner mask_result (agg.py:284-318): fix_precision(val) + seed_mask + sum(+-mask).
    k = 16 fills one launch's generator slots (the full 64-KB dynamic LDS);
    k = 19 takes two launches."""
    rng = np.random.default_rng(3)
    val = rng.standard_normal((37, 129)) * 100
    seeds = [os.urandom(32) for _ in range(k)]
    signs = [1] + [(-1) ** i for i in range(k - 1)]
    terms = list(zip(seeds, signs))
    got = utils.masked_sum(torch.from_numpy(val), terms, precision=8).cpu().numpy()
    want = pm.fix_precision(val, 8)
    for s, sg in terms:
        want = want + sg * pm.make_mask_numpy(s, val.shape)
    assert np.array_equal(got, want)
    # coordinator inverse: subtract them all, unfix
    back = utils.unmasked_values(torch.from_numpy(got), [(s, -sg) for s, sg in terms], 8).cpu().numpy()
    assert np.array_equal(back, pm.unfix_precision(pm.fix_precision(val, 8), 8))


def test_reference_test_calc_restated():
    """tests/utils_test.py:44-62 of the reference, with random pairwise keys
    standing in for the ECDH shared keys: the masked sum of 3 clients minus
    their seed masks averages to the plain mean."""
    arrs = [np.random.random(10) for _ in range(3)]
    seeds = [os.urandom(32) for _ in range(3)]
    pair = {(i, j): os.urandom(32) for i in range(3) for j in range(3) if i < j}
    key = lambda i, j: pair[(min(i, j), max(i, j))]  # noqa: E731
    masked = []
    for i in range(3):
        terms = [(seeds[i], 1)] + [(key(i, j), -1 if i < j else 1) for j in range(3) if j != i]
        masked.append(utils.masked_sum(torch.from_numpy(arrs[i]), terms, precision=8))
    total = masked[0] + masked[1] + masked[2]
    res = utils.unmasked_values(total, [(s, -1) for s in seeds], 8).cpu().numpy()
    assert np.allclose(res / 3, np.mean(arrs, 0))


def test_exact_replay_on_rejections():
    """A range where Lemire rejects a quarter of the raw draws exercises the
    exact replay (per-segment raw offsets) against numpy."""
    seed = bytes(range(32))
    low, high = -3 * 2**61, 3 * 2**61
    for n in (1, 100, 5000, 100003):
        got = bounded_sum([(seed, 1)], n, low, high).cpu().numpy()
        ref = np.random.default_rng(list(seed)).integers(low, high, size=n, dtype=np.int64)
        assert np.array_equal(got, ref), n
    # two generators, one subtracted, with a base
    s2 = os.urandom(32)
    base = torch.arange(20000, dtype=torch.int64, device="cuda")
    got = bounded_sum([(seed, 1), (s2, -1)], 20000, low, high, base_i64=base).cpu().numpy()
    r1 = np.random.default_rng(list(seed)).integers(low, high, size=20000, dtype=np.int64)
    r2 = np.random.default_rng(list(s2)).integers(low, high, size=20000, dtype=np.int64)
    assert np.array_equal(got, np.arange(20000, dtype=np.int64) + r1 - r2)
    # the subtracted generator listed first: the kernel sorts generators by
    # sign, so its reject flags must map back to the caller's order
    got = bounded_sum([(s2, -1), (seed, 1)], 20000, low, high, base_i64=base).cpu().numpy()
    assert np.array_equal(got, np.arange(20000, dtype=np.int64) + r1 - r2)
    s3 = os.urandom(32)
    r3 = np.random.default_rng(list(s3)).integers(low, high, size=20000, dtype=np.int64)
    got = bounded_sum([(s2, -1), (s3, -1), (seed, 1)], 20000, low, high).cpu().numpy()
    assert np.array_equal(got, r1 - r2 - r3)


def test_fix_unfix_precision_match_numpy_semantics():
    got = utils.fix_precision(Z["fix_in"], 8)
    assert np.array_equal(got, Z["fix8"])  # includes NaN / inf / out of range -> INT64_MIN
    assert np.array_equal(utils.unfix_precision(Z["unfix_in"], 8), Z["unfix8"])
    x = np.random.default_rng(1).standard_normal((5, 6)).astype(np.float32)
    assert np.array_equal(utils.fix_precision(x, 3), pm.fix_precision(x, 3))


def test_raw_offsets_and_ranges():
    """Segment API: elements [b, e) drawing raw e + k equal numpy's stream shifted by k."""
    seed = os.urandom(32)
    g = mn.pcg64(seed)
    n = 9000
    ref = np.random.default_rng(list(seed)).integers(0, 2**47 - 1, size=n + 50, dtype=np.int64)
    out = torch.zeros(n, dtype=torch.int64, device="cuda")
    mn.accumulate([g], [1], out, n, 0, 2**47 - 2, raw_offsets=[37], elem_begin=1234, elem_end=8000)
    o = out.cpu().numpy()
    assert np.array_equal(o[1234:8000], ref[1234 + 37:8000 + 37])
    assert not o[:1234].any() and not o[8000:].any()


@pytest.mark.parametrize("grid", [None, "1"])
def test_small_tile_kernel_matches(grid, monkeypatch):
    """The small-tile accumulate (DN_MASK_SMALL, csrc/mask_pcg64.hip: 512-element
    tiles, generator states in registers stepped tile to tile by T^(nwaves 512))
    through the tuning build: the reference's fixture and 2^24 digests, signed
    sums of 12 / 16 / 19 generators, the exact replay on rejections and the
    segment API — with the default resident grid and with one workgroup per CU
    (every wave stepping through many tiles)."""
    from delta_node.crypto.shamir import _native

    monkeypatch.setenv("DN_MASK_SMALL", "1")
    if grid:
        monkeypatch.setenv("DN_MASK_GRID", grid)
    with _native.library(_native.TUNING_LIB):
        test_make_mask_matches_reference_fixture()
        test_make_mask_digests_up_to_2e24()
        for n in (1, 511, 513, 70001):
            test_make_mask_ragged_vs_numpy(n)
        for k in (12, 16, 19):
            test_masked_sum_matches_reference_composition(k)
        test_exact_replay_on_rejections()
        test_raw_offsets_and_ranges()
