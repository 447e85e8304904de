"""Pin the CPU oracle (oracle/) to the reference's own outputs (tests/golden/).

CPU only.  The golden fixtures were generated from the real reference
(delta_node/crypto/shamir/shamir.py) by tests/golden/make_golden.py; here the
two restatements — pure Python (oracle/py_shamir.py) and plain C
(oracle/m521_oracle.c) — must reproduce them bit for bit before the GPU tests
may use them as checkers.
"""
import random

import numpy as np
import pytest

from golden.fixtures import (P, combine_digests, chunk_digests, ints_to_limbs, limbs_to_ints, load_json, load_npz,
                             manifest, secrets_int64, unpack_share_bytes)
from oracle import c_oracle
from oracle.py_shamir import RefSecretShare, parse_share

MASK64 = (1 << 64) - 1


def u64_bytes(v):
    return (int(v) & MASK64).to_bytes(8, "big")


@pytest.fixture(scope="module")
def man():
    return manifest()


@pytest.mark.parametrize("key", ["f1", "f2"])
def test_py_oracle_vector_fixture(man, key):
    cfg = man[key]
    z = load_npz(cfg["file"])
    ss = RefSecretShare(cfg["t"], seed=cfg["mt_seed"])
    flat, offs = z["share_bytes"], z["share_offsets"]
    n = cfg["n"]
    for e, v in enumerate(z["secrets"]):
        shares = ss.make_shares(u64_bytes(v), n)
        for x in range(n):
            assert shares[x] == unpack_share_bytes(flat, offs, e * n + x)
    for sub, size in zip(z["recon_subsets"], z["recon_sizes"]):
        xs = [int(x) for x in sub[:size]]
        for e in range(0, cfg["N"], 37):
            got = ss.resolve_shares([unpack_share_bytes(flat, offs, e * n + x - 1) for x in xs])
            assert got == (int(z["secrets"][e]) & MASK64).to_bytes(8, "big").lstrip(b"\x00")


def test_py_oracle_edge_fixture():
    f3 = load_json("f3_edge.json")
    for case in f3["cases"]:
        if case["n"] > 9:  # the long cases are covered by the C oracle / GPU tests
            continue
        ss = RefSecretShare(case["t"], seed=case["mt_seed"])
        shares = ss.make_shares(bytes.fromhex(case["value"]), case["n"])
        assert [s.hex() for s in shares] == case["shares"]
        for r in case["resolve"]:
            sh = [shares[x - 1] for x in r["xs"]]
            if "exc" in r:
                with pytest.raises(Exception) as ei:
                    ss.resolve_shares(sh)
                assert type(ei.value).__name__ == r["exc"] and str(ei.value) == r["msg"]
            else:
                assert ss.resolve_shares(sh).hex() == r["out"]


def test_py_oracle_errors():
    f3 = load_json("f3_edge.json")
    msgs = {(e["call"], e["arg"]): (e["exc"], e.get("msg")) for e in f3["errors"]}
    ss = RefSecretShare(4)
    with pytest.raises(ValueError, match="threshold should be little equal than shares"):
        ss.make_shares(b"\x01", 3)
    assert msgs[("make", 3)] == ("ValueError", "threshold should be little equal than shares")
    with pytest.raises(ValueError) as ei:
        ss.resolve_shares(RefSecretShare(4).make_shares(b"\x05", 6)[:2])
    assert (type(ei.value).__name__, str(ei.value)) == msgs[("resolve", 2)]
    with pytest.raises(ValueError) as ei:
        ss.resolve_shares([])
    assert (type(ei.value).__name__, str(ei.value)) == msgs[("resolve", 0)]
    sh = RefSecretShare(4).make_shares(b"\x05", 6)
    with pytest.raises(ValueError) as ei:
        ss.resolve_shares([sh[0], sh[1], sh[2], sh[1]])
    assert (type(ei.value).__name__, str(ei.value)) == msgs[("dup", None)]


def test_py_oracle_recon_fixture():
    for group in load_json("f4_recon.json"):
        xs = group["xs"]
        ss = RefSecretShare(len(xs))
        for row in group["rows"]:
            ys = [int(y, 16) for y in row["ys"]]
            sh = [bytes([len(x.to_bytes((x.bit_length() + 7) // 8, "big"))]) + x.to_bytes((x.bit_length() + 7) // 8, "big")
                  + y.to_bytes((y.bit_length() + 7) // 8, "big") for x, y in zip(xs, ys)]
            if "exc" in row:
                with pytest.raises(Exception) as ei:
                    ss.resolve_shares(sh)
                assert type(ei.value).__name__ == row["exc"]
            else:
                assert ss.resolve_shares(sh).hex() == row["out"]


def test_c_oracle_mt_stream():
    for seed in (0, 1, 1234, 2**32 + 5):
        r = random.Random(seed)
        want = np.array([r.getrandbits(32) for _ in range(2000)], dtype=np.uint32)
        assert np.array_equal(c_oracle.mt_words(seed, 2000), want)


@pytest.mark.parametrize("key", ["f1", "f2"])
def test_c_oracle_vector_fixture(man, key):
    cfg = man[key]
    z = load_npz(cfg["file"])
    co = c_oracle.draw_coeffs(cfg["mt_seed"], cfg["N"], cfg["t"] - 1)
    assert np.array_equal(co, z["coeff_limbs"])
    sh = c_oracle.split(z["secrets"], co, cfg["t"], cfg["n"])  # [n, N, 17]
    assert np.array_equal(sh.transpose(1, 0, 2), z["share_limbs"])
    for sub, size in zip(z["recon_subsets"], z["recon_sizes"]):
        xs = [int(x) for x in sub[:size]]
        out = c_oracle.reconstruct(sh[[x - 1 for x in xs]], xs)
        assert np.array_equal(out[:, 2:], np.zeros_like(out[:, 2:]))
        got = out[:, 0].astype(np.uint64) | (out[:, 1].astype(np.uint64) << np.uint64(32))
        assert np.array_equal(got, z["secrets"].view(np.uint64))


def test_c_oracle_recon_fixture():
    for group in load_json("f4_recon.json"):
        xs = group["xs"]
        if len(xs) > 16 or max(xs) > 1000 or len(xs) < 2:
            continue
        rows = [r for r in group["rows"] if "out" in r and all(int(y, 16) < (1 << 544) for y in r["ys"])]
        ys = np.stack([ints_to_limbs([int(r["ys"][i], 16) for r in rows]) for i in range(len(xs))])
        out = limbs_to_ints(c_oracle.reconstruct(ys, xs))
        assert out == [int(r["out"], 16) if r["out"] else 0 for r in rows]


def test_c_oracle_edge_fixture_splits():
    """Long edge cases (n up to 300) through the C oracle with the recorded coefficients."""
    f3 = load_json("f3_edge.json")
    for case in f3["cases"]:
        value = int(case["value"], 16) if case["value"] else 0
        if value >= (1 << 64):
            continue  # the C oracle's split takes u64 secrets (the vector path)
        t, n = case["t"], case["n"]
        co = ints_to_limbs([int(c, 16) for c in case["coeffs"]]).reshape(1, t - 1, 17) if t > 1 else \
            np.zeros((1, 0, 17), np.uint32)
        sh = c_oracle.split(np.array([value], dtype=np.uint64).view(np.int64), co, t, n)
        ys = limbs_to_ints(sh[:, 0, :])
        assert [parse_share(bytes.fromhex(s))[1] for s in case["shares"]] == ys


def _digest_split_c(d):
    N = d["N"]
    sec = secrets_int64(d["secret_seed"], N)
    co = c_oracle.draw_coeffs(d["mt_seed"], N, d["t"] - 1)
    sh = c_oracle.split(sec, co, d["t"], d["n"])  # [n, N, 17]
    return combine_digests(chunk_digests(np.ascontiguousarray(sh.transpose(0, 2, 1))))


def test_c_oracle_split_digests(man):
    for d in man["digests"]:
        if d["kind"] == "split" and d["N"] <= (1 << 16):
            assert _digest_split_c(d) == d["digest"], d["name"]


def test_c_oracle_recon_digests(man):
    for d in man["digests"]:
        if d["kind"] != "recon" or d["N"] > (1 << 16):
            continue
        k = len(d["xs"])
        ys = c_oracle.draw_coeffs(d["mt_seed"], d["N"], k).transpose(1, 0, 2)  # [k, N, 17]
        assert combine_digests(chunk_digests(np.ascontiguousarray(ys.transpose(0, 2, 1)))) == d["input_digest"]
        out = c_oracle.reconstruct(ys, d["xs"])
        assert combine_digests(chunk_digests(np.ascontiguousarray(out.T[None]))) == d["digest"], d["name"]
