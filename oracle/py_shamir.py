"""Pure-Python restatement of delta_node/crypto/shamir — TEST INFRASTRUCTURE ONLY.

The reference is pure Python (Python ints, stdlib MT19937), so its algorithm is
restated here with the same int semantics, one element per call:

  PRIME                    shamir.py:16
  eval_at                  shamir.py:19-25   (Horner from the top, % p each step)
  share_to_bytes / parse   shamir.py:28-45   ([len(x)][x][y], minimal big-endian)
  RefSecretShare           shamir.py:48-90   (make_shares / resolve_shares)
  _inv                     op.py:4-25        (extended Euclid; same asserts)

Used for small parity cases, as the pinned checker of the C oracle, and as
bench.py's cpu_baseline ("port", 1 core).  Pinned by tests/golden (outputs of
the reference itself): tests/test_oracle.py.
"""
from __future__ import annotations

import random
from typing import List, Sequence, Tuple

PRIME = (1 << 521) - 1


def int_to_bytes(v: int) -> bytes:
    return v.to_bytes((v.bit_length() + 7) // 8, "big")


def eval_at(coeffs: Sequence[int], x: int, p: int = PRIME) -> int:
    acc = 0
    for c in reversed(coeffs):
        acc = (acc * x + c) % p
    return acc


def share_to_bytes(x: int, y: int) -> bytes:
    xb = int_to_bytes(x)
    return bytes([len(xb)]) + xb + int_to_bytes(y)


def parse_share(data: bytes) -> Tuple[int, int]:
    n = data[0] if data else 0
    return int.from_bytes(data[1:1 + n], "big"), int.from_bytes(data[1 + n:], "big")


def _egcd(a: int, b: int):
    x0, x1, y0, y1 = 1, 0, 0, 1
    while b:
        q = a // b
        a, b = b, a - q * b
        x0, x1 = x1, x0 - q * x1
        y0, y1 = y1, y0 - q * y1
    return a, x0, y0


def _inv(k: int, p: int) -> int:
    if k == 0:
        raise ZeroDivisionError
    g, s, _ = _egcd(k, p)
    assert g == 1 and (k * s) % p == 1
    return s % p


def _prod(vals: List[int]) -> int:
    if not vals:
        raise TypeError("reduce() of empty iterable with no initial value")
    out = 1
    for v in vals:
        out *= v
    return out


class RefSecretShare:
    """Per-element restatement of the reference `SecretShare`."""

    def __init__(self, threshold: int, p: int = PRIME, seed=None):
        self.threshold = threshold
        self.prime = p
        self.random = random.Random(seed)

    def coefficients(self, value: bytes) -> List[int]:
        head = int.from_bytes(value, "big")
        return [head] + [self.random.randint(1, self.prime - 1) for _ in range(self.threshold - 1)]

    def make_shares(self, value: bytes, shares: int) -> List[bytes]:
        if self.threshold > shares:
            raise ValueError("threshold should be little equal than shares")
        cs = self.coefficients(value)
        return [share_to_bytes(x, eval_at(cs, x, self.prime)) for x in range(1, shares + 1)]

    def resolve_shares(self, shares: List[bytes]) -> bytes:
        pts = [parse_share(s) for s in shares]
        if not pts:
            raise ValueError("not enough values to unpack (expected 2, got 0)")
        xs = [x for x, _ in pts]
        ys = [y for _, y in pts]
        k, p = len(xs), self.prime
        if k < self.threshold:
            raise ValueError("need at least {} shares".format(self.threshold))
        if len(set(xs)) != k:
            raise ValueError("shares must be distinct")
        nums = [_prod([-xs[j] for j in range(k) if j != i]) for i in range(k)]
        dens = [_prod([xs[i] - xs[j] for j in range(k) if j != i]) for i in range(k)]
        den = _prod(dens)
        total = 0
        for i in range(k):
            total += (nums[i] * den * ys[i] % p) * _inv(dens[i], p) % p
        return int_to_bytes(total * _inv(den, p) % p)


def time_elements(t: int, n: int, xs: Sequence[int], budget_s: float, seed: int, max_elems: int = 1 << 22):
    """bench.py's cpu_baseline leg: per element make_shares + resolve_shares
    (checked) over int64 secrets from numpy PCG64(seed) until `budget_s`
    seconds have passed.  Returns (elements done, seconds)."""
    import time

    import numpy as np

    ss = RefSecretShare(t, seed=seed)
    sec = np.random.default_rng(seed).integers(-(1 << 63), (1 << 63) - 1, size=max_elems, endpoint=True,
                                               dtype=np.int64)
    done = 0
    t0 = time.perf_counter()
    while done < max_elems:
        v = int(sec[done]) & ((1 << 64) - 1)
        shares = ss.make_shares(v.to_bytes(8, "big"), n)
        out = ss.resolve_shares([shares[x - 1] for x in xs])
        assert int.from_bytes(out, "big") == v
        done += 1
        if (done & 255) == 0 and time.perf_counter() - t0 > budget_s:
            break
    return done, time.perf_counter() - t0


def time_elements_star(args):
    return time_elements(*args)
