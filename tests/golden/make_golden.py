#!/usr/bin/env python3
"""Generate the golden fixtures from the REAL reference (build container only).

    python tests/golden/make_golden.py            # small fixtures + 2^16/2^20 digests
    python tests/golden/make_golden.py --big      # adds the 2^24 split digest (~5 min)
    python tests/golden/make_golden.py --only recon_135_2e24,recon_245_2e24,split_t5n9_2e22
                                                  # just the named full-size digests, one
                                                  # process each, merged into manifest.json

The reference `delta_node/crypto/shamir/shamir.py` is loaded by file path
(`_ref_loader.py`); every expected value below is an output of the reference's
own `SecretShare.make_shares` (shamir.py:55-66) / `resolve_shares`
(shamir.py:68-90).  Coefficients are observed, not re-derived: the instance's
`random` attribute is replaced by a seeded `random.Random` subclass that records
each `randint` result the reference draws (shamir.py:59-61), so the fixtures
pin both the share values and the MT19937 coefficient stream.

Outputs (all small, committed): manifest.json, f1_t3n5.npz, f2_t5n9.npz,
f3_edge.json, f4_recon.json.  The reference never leaves this container.
"""
from __future__ import annotations

import argparse
import itertools
import json
import os
import random
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

from _ref_loader import load_reference_shamir  # noqa: E402
from fixtures import (P, chunk_digests, combine_digests, ints_to_limbs,  # noqa: E402
                      secrets_int64)

ref = load_reference_shamir()
assert ref.PRIME == P
MASK64 = (1 << 64) - 1


class RecordingRandom(random.Random):
    """random.Random that records the values `randint` hands to the reference."""

    def __init__(self, seed):
        super().__init__(seed)
        self.drawn = []

    def randint(self, a, b):  # same stream as random.Random.randint
        v = super().randint(a, b)
        self.drawn.append(v)
        return v


def u64_bytes(v: int) -> bytes:
    return (int(v) & MASK64).to_bytes(8, "big")


def parse_y(share: bytes) -> int:
    xl = share[0]
    return int.from_bytes(share[1 + xl:], "big")


def vector_fixture(name, t, n, N, secret_seed, mt_seed, subsets):
    ss = ref.SecretShare(t)
    ss.random = RecordingRandom(mt_seed)
    secrets = secrets_int64(secret_seed, N)
    flat, offsets, ys = [], [0], []
    for v in secrets:
        shares = ss.make_shares(u64_bytes(v), n)
        for s in shares:
            flat.append(s)
            offsets.append(offsets[-1] + len(s))
            ys.append(parse_y(s))
    coeffs = ss.random.drawn
    assert len(coeffs) == N * (t - 1)
    recon = []
    for sub in subsets:
        out = []
        for e in range(N):
            sh = [flat[e * n + (x - 1)] for x in sub]
            out.append(ss.resolve_shares(sh))
        recon.append(out)
        for e in range(N):
            assert out[e] == ref.serialize.int_to_bytes(int(secrets[e]) & MASK64)
    np.savez_compressed(
        os.path.join(HERE, name),
        secrets=secrets,
        share_bytes=np.frombuffer(b"".join(flat), dtype=np.uint8),
        share_offsets=np.array(offsets, dtype=np.int64),
        share_limbs=ints_to_limbs(ys).reshape(N, n, 17),
        coeff_limbs=ints_to_limbs(coeffs).reshape(N, t - 1, 17) if t > 1 else np.zeros((N, 0, 17), np.uint32),
        recon_subsets=np.array([list(s) + [0] * (n - len(s)) for s in subsets], dtype=np.int64),
        recon_sizes=np.array([len(s) for s in subsets], dtype=np.int64),
    )
    return {"file": name, "t": t, "n": n, "N": N, "secret_seed": secret_seed, "mt_seed": mt_seed,
            "subsets": [list(s) for s in subsets]}


def edge_fixture():
    cases = []
    values = [
        b"", b"\x00", b"\x00\x01", b"\x01", b"\xff" * 8, b"\x80" + b"\x00" * 7,
        bytes(range(32)), b"\xff" * 32,
        P.to_bytes(66, "big"), (P - 1).to_bytes(66, "big"), (P + 5).to_bytes(66, "big"),
        (1 << 527).to_bytes(66, "big"), b"\xab" * 100,
    ]
    params = [(1, 1), (1, 3), (2, 5), (3, 5), (5, 9), (4, 4), (3, 255), (2, 256), (2, 300)]
    seed = 7
    for value in values:
        for (t, n) in params:
            seed += 1
            ss = ref.SecretShare(t)
            ss.random = RecordingRandom(seed)
            shares = ss.make_shares(value, n)
            rec = []
            subsets = [list(range(1, n + 1))]
            if n > t:
                subsets.append(list(range(n, n - t, -1)))
                subsets.append([1] + list(range(n - t + 2, n + 1)))
            for sub in subsets:
                try:
                    rec.append({"xs": sub, "out": ss.resolve_shares([shares[x - 1] for x in sub]).hex()})
                except Exception as e:  # noqa: BLE001 — e.g. k == 1: reduce() of empty iterable
                    rec.append({"xs": sub, "exc": type(e).__name__, "msg": str(e)})
            cases.append({"value": value.hex(), "t": t, "n": n, "mt_seed": seed,
                          "coeffs": [hex(c) for c in ss.random.drawn],
                          "shares": [s.hex() for s in shares], "resolve": rec})
    errors = []
    ss = ref.SecretShare(4)
    for call in [("make", b"\x01", 3), ("resolve", 2), ("resolve", 0), ("dup", None)]:
        try:
            if call[0] == "make":
                ss.make_shares(call[1], call[2])
            elif call[0] == "resolve":
                sh = ref.SecretShare(4).make_shares(b"\x05", 6)[:call[1]]
                ss.resolve_shares(sh)
            else:
                sh = ref.SecretShare(4).make_shares(b"\x05", 6)
                ss.resolve_shares([sh[0], sh[1], sh[2], sh[1]])
            errors.append({"call": call[0], "arg": call[-1], "exc": None})
        except Exception as e:  # noqa: BLE001 — recording the reference's error behaviour
            errors.append({"call": call[0], "arg": call[-1] if call[0] != "dup" else None,
                           "exc": type(e).__name__, "msg": str(e)})
    return {"cases": cases, "errors": errors}


def recon_fixture():
    """Inconsistent (random-y) shares: reference output = Lagrange interpolant at 0."""
    rng = random.Random(2024)
    sets = [[1, 2, 3], [1, 3, 5], [2, 4, 5], [3, 4, 5], [5, 1, 3], [1, 2, 4, 5], [1, 2, 3, 4, 5],
            [1, 3, 5, 7, 9], [2, 3, 5, 8, 9], [7, 100, 255], [1, 256, 1000], [2, 3],
            [1, 2, 3, 4, 5, 6, 7, 8, 9], [9, 8, 7, 6, 5, 4, 3, 2, 1], [4], [17, 33, 65, 129, 200, 250]]
    out = []
    for xs in sets:
        k = len(xs)
        ss = ref.SecretShare(k)
        rows = []
        specials = [[0] * k, [P - 1] * k, [1] * k, [P] * k, [(1 << 528) + 3] * k]
        for i in range(48):
            ys = [rng.randrange(P) for _ in range(k)]
            rows.append(ys)
        rows.extend(specials)
        res = []
        for ys in rows:
            shares = [ref._share_to_bytes((x, y)) for x, y in zip(xs, ys)]
            try:
                res.append({"ys": [hex(y) for y in ys], "out": ss.resolve_shares(shares).hex()})
            except Exception as e:  # noqa: BLE001
                res.append({"ys": [hex(y) for y in ys], "exc": type(e).__name__, "msg": str(e)})
        out.append({"xs": xs, "rows": res})
    return out


def split_digest(t, n, N, secret_seed, mt_seed, log=True):
    ss = ref.SecretShare(t)
    ss.random.seed(mt_seed)
    secrets = secrets_int64(secret_seed, N)
    chunks = []
    t0 = time.time()
    C = 1 << 16
    for lo in range(0, N, C):
        hi = min(N, lo + C)
        ys = []
        for v in secrets[lo:hi]:
            ys.extend(parse_y(s) for s in ss.make_shares(u64_bytes(v), n))
        limbs = ints_to_limbs(ys).reshape(hi - lo, n, 17).transpose(1, 2, 0)  # [n,17,chunk]
        chunks.extend(chunk_digests(np.ascontiguousarray(limbs), threads=1))
        if log and (lo // C) % 16 == 0:
            print(f"  split t{t}n{n} N={N}: {hi}/{N} elements, {time.time() - t0:.0f}s", flush=True)
    return {"kind": "split", "t": t, "n": n, "N": N, "secret_seed": secret_seed, "mt_seed": mt_seed,
            "digest": combine_digests(chunks)}


def recon_digest(xs, N, mt_seed):
    """y values = the MT stream of randint(1, p-1), element-major (k per element)."""
    k = len(xs)
    r = random.Random(mt_seed)
    ss = ref.SecretShare(k)
    chunks_in, chunks_out = [], []
    C = 1 << 16
    for lo in range(0, N, C):
        hi = min(N, lo + C)
        ys_all, outs = [], []
        for _ in range(lo, hi):
            ys = [r.randint(1, P - 1) for _ in range(k)]
            ys_all.extend(ys)
            shares = [ref._share_to_bytes((x, y)) for x, y in zip(xs, ys)]
            outs.append(int.from_bytes(ss.resolve_shares(shares), "big"))
        limbs_in = ints_to_limbs(ys_all).reshape(hi - lo, k, 17).transpose(1, 2, 0)
        limbs_out = ints_to_limbs(outs).reshape(hi - lo, 1, 17).transpose(1, 2, 0)
        chunks_in.extend(chunk_digests(np.ascontiguousarray(limbs_in), threads=1))
        chunks_out.extend(chunk_digests(np.ascontiguousarray(limbs_out), threads=1))
    return {"kind": "recon", "xs": xs, "N": N, "mt_seed": mt_seed,
            "input_digest": combine_digests(chunks_in), "digest": combine_digests(chunks_out)}


# Full-size pins of BASELINE configs 2-4 (one reference process each, minutes).
BIG_DIGESTS = {
    "split_t3n5_2e24": lambda: split_digest(3, 5, 1 << 24, 1, 1),
    # config 3: reconstruct of 2^24 elements from random (inconsistent) share
    # values, the same element-major MT stream as the 2^18 digests
    "recon_135_2e24": lambda: recon_digest([1, 3, 5], 1 << 24, 31),
    "recon_245_2e24": lambda: recon_digest([2, 4, 5], 1 << 24, 32),
    # config 4's 5-of-9 split at 2^22 (2^26 would take the reference ~1.5 h)
    "split_t5n9_2e22": lambda: split_digest(5, 9, 1 << 22, 13, 3),
}


def _run_big(name):
    t0 = time.time()
    d = BIG_DIGESTS[name]()
    d["name"] = name
    print(f"{name} done {time.time() - t0:.1f}s", flush=True)
    return d


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--big", action="store_true", help="also the 2^24 split digest")
    ap.add_argument("--only", default="", help="comma-separated BIG_DIGESTS names; nothing else")
    args = ap.parse_args()
    path = os.path.join(HERE, "manifest.json")
    man = json.load(open(path)) if os.path.exists(path) else {}
    if args.only:
        import multiprocessing as mp
        names = args.only.split(",")
        with mp.get_context("fork").Pool(len(names)) as pool:
            new = pool.map(_run_big, names)
        digests = {d["name"]: d for d in man.get("digests", [])}
        digests.update({d["name"]: d for d in new})
        man["digests"] = sorted(digests.values(), key=lambda d: d["name"])
        json.dump(man, open(path, "w"), indent=1)
        print("wrote", path)
        return
    man["generator"] = "tests/golden/make_golden.py (reference delta_node/crypto/shamir loaded by file path)"
    man["python"] = sys.version.split()[0]
    t0 = time.time()
    man["f1"] = vector_fixture("f1_t3n5.npz", 3, 5, 1024, 0, 1234,
                               [(1, 2, 3), (1, 3, 5), (2, 4, 5), (5, 4, 3), (1, 2, 3, 4), (1, 2, 3, 4, 5)])
    man["f2"] = vector_fixture("f2_t5n9.npz", 5, 9, 256, 2, 99,
                               [(1, 3, 5, 7, 9), (2, 3, 5, 8, 9), (1, 2, 3, 4, 5, 6, 7, 8, 9)])
    print(f"f1/f2 done {time.time() - t0:.1f}s", flush=True)
    json.dump(edge_fixture(), open(os.path.join(HERE, "f3_edge.json"), "w"))
    json.dump(recon_fixture(), open(os.path.join(HERE, "f4_recon.json"), "w"))
    print(f"f3/f4 done {time.time() - t0:.1f}s", flush=True)
    digests = {d["name"]: d for d in man.get("digests", [])}
    for name, fn in [
        ("split_t3n5_2e16", lambda: split_digest(3, 5, 1 << 16, 11, 1)),
        ("split_t5n9_2e16", lambda: split_digest(5, 9, 1 << 16, 12, 2)),
        ("recon_245_2e18", lambda: recon_digest([2, 4, 5], 1 << 18, 21)),
        ("recon_135_2e18", lambda: recon_digest([1, 3, 5], 1 << 18, 22)),
        ("recon_13579_2e16", lambda: recon_digest([1, 3, 5, 7, 9], 1 << 16, 23)),
    ]:
        d = fn()
        d["name"] = name
        digests[name] = d
        print(f"{name} done {time.time() - t0:.1f}s", flush=True)
    if args.big:
        digests["split_t3n5_2e24"] = _run_big("split_t3n5_2e24")
    man["digests"] = sorted(digests.values(), key=lambda d: d["name"])
    json.dump(man, open(path, "w"), indent=1)
    print("wrote", path)


if __name__ == "__main__":
    main()
