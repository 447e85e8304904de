"""Modular helpers of the reference (delta_node/crypto/shamir/op.py:4-29).

Host-side integer helpers (Lagrange constants are computed once per call, not
per element).  Same results and exceptions as the reference:
`inverse_mod(0, p)` raises ZeroDivisionError; a non-invertible k fails the
gcd assertion.
"""
from typing import Tuple

__all__ = ["extend_gcd", "inverse_mod", "div_mod"]


def extend_gcd(a: int, b: int) -> Tuple[int, int, int]:
    """(g, s, t) with a*s + b*t == g == gcd(a, b): iterative Euclid (op.py:4-13)."""
    r0, r1 = a, b
    s0, s1 = 1, 0
    t0, t1 = 0, 1
    while r1:
        q, rem = divmod(r0, r1)
        r0, r1 = r1, rem
        s0, s1 = s1, s0 - q * s1
        t0, t1 = t1, t0 - q * t1
    return r0, s0, t0


def inverse_mod(k: int, p: int) -> int:
    """k^-1 mod p (op.py:16-25)."""
    if k == 0:
        raise ZeroDivisionError
    g, s, _ = extend_gcd(k, p)
    assert g == 1
    assert (k * s) % p == 1
    return s % p


def div_mod(a: int, b: int, p: int) -> int:
    """a / b mod p (op.py:28-29)."""
    return (a * inverse_mod(b, p)) % p
