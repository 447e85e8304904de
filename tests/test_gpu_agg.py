"""Coordinator masked-result sum and an end-to-end
secure-aggregation round through every row built so far.

make_masked_results (coord/horizontal/agg.py:227-251) is restated with numpy
`+=` as the checker; the round follows runner/horizontal/agg.py:137-318 and
coord/horizontal/agg.py:274-406 with random pairwise keys in place of the
ECDH shared keys (OpenSSL, out of scope).  Bit-exact integers; the final
float mean within the reference test's np.allclose (tests/utils_test.py:62).
"""
import os

import numpy as np
import pytest
import torch

from delta_node import utils
from delta_node.crypto import shamir

pytestmark = pytest.mark.gpu


def _ref_make_masked_results(members, agg_vars):
    result, valid = {}, []
    for i, res in enumerate(members):
        names = res.keys()
        if len(names) == len(agg_vars) and len(set(names) - set(agg_vars)) == 0:
            valid.append(i)
            for var in names:
                result.setdefault(var, {})
                for key, val in res[var].items():
                    if key in result[var]:
                        result[var][key] = result[var][key] + val
                    else:
                        result[var][key] = val.copy()
    return valid, result


@pytest.mark.parametrize("k", [1, 2, 3, 5, 8, 9, 10, 16, 17, 40])
def test_sum_member_results_matches_reference(k):
    rng = np.random.default_rng(k)
    shapes = {"w": {"a": (33, 7), "b": (1,)}, "v": {"c": (1001,)}}
    members = []
    for i in range(k):
        m = {var: {key: rng.integers(-2**63, 2**63 - 1, size=shp, dtype=np.int64, endpoint=True)
                   for key, shp in keys.items()} for var, keys in shapes.items()}
        if i % 7 == 3:
            m = {"w": m["w"]}  # invalid: missing a variable
        members.append(m)
    valid, got = utils.sum_member_results(members, ["w", "v"])
    rvalid, want = _ref_make_masked_results(members, ["w", "v"])
    assert valid == rvalid
    for var in want:
        for key in want[var]:
            assert np.array_equal(got[var][key].cpu().numpy(), want[var][key]), (var, key)


def test_secure_aggregation_round_end_to_end():
    """5 clients, threshold 3: each Shamir-shares its mask seed (vector path not
    needed: 32-byte seeds, byte API), masks its result with the seed mask and
    pairwise masks, the coordinator sums the masked results, reconstructs the
    seeds from 3 shares each and unmasks.  The pairwise masks cancel."""
    n_clients, t = 5, 3
    rng = np.random.default_rng(0)
    results = [rng.standard_normal((64, 33)) for _ in range(n_clients)]
    seeds = [bytes([1]) + os.urandom(31) for _ in range(n_clients)]  # non-zero lead byte: survives int_to_bytes
    pair = {(i, j): os.urandom(32) for i in range(n_clients) for j in range(i + 1, n_clients)}
    ss = shamir.SecretShare(t)
    seed_shares = [ss.make_shares(s, n_clients) for s in seeds]  # runner/horizontal/agg.py:142-144
    masked = []
    for i in range(n_clients):
        terms = [(seeds[i], 1)]
        for j in range(n_clients):
            if j != i:
                terms.append((pair[(min(i, j), max(i, j))], -1 if i < j else 1))  # agg.py:301-306
        masked.append({"w": {"k": utils.masked_sum(torch.from_numpy(results[i]), terms, precision=8)}})
    valid, summed = utils.sum_member_results(masked, ["w"])
    assert valid == list(range(n_clients))
    recovered = [ss.resolve_shares([seed_shares[i][x] for x in (0, 2, 4)]) for i in range(n_clients)]
    assert recovered == seeds
    mean = utils.unmasked_values(summed["w"]["k"], [(s, -1) for s in recovered], 8).cpu().numpy() / n_clients
    assert np.allclose(mean, np.mean(results, 0))
    # bit-exact: the unmasked integer sum equals the sum of fixed-point inputs
    ints = utils.masked_sum(summed["w"]["k"], [(s, -1) for s in recovered]).cpu().numpy()
    assert np.array_equal(ints, np.sum([utils.fix_precision(r, 8) for r in results], axis=0))
