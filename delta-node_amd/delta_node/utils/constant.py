"""BN254 / MiMC7 field parameters (reference: delta_node/utils/constant.py:1-30).

Same names and values: q(), data_block_size(), cts().  The numbers are read
from the library that computes with them (dn_mimc7_params, csrc/host_mimc7.cpp;
defined once in csrc/mimc7_consts.hpp for the device kernels and the host
chain), so the Python view can never drift from what the kernels use.
"""
from __future__ import annotations

import ctypes
import functools
from typing import List, Tuple

__all__ = ["q", "data_block_size", "cts"]


@functools.lru_cache(maxsize=1)
def _params() -> Tuple[int, Tuple[int, ...]]:
    from ..crypto.shamir import _native

    L = _native.lib()
    qb = (ctypes.c_uint32 * 8)()
    cb = (ctypes.c_uint32 * (13 * 8))()
    L.dn_mimc7_params.restype = ctypes.c_int
    L.dn_mimc7_params.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    _native.check(L.dn_mimc7_params(ctypes.addressof(qb), ctypes.addressof(cb)))
    q_int = int.from_bytes(bytes(qb), "little")
    raw = bytes(cb)
    cts_int = tuple(int.from_bytes(raw[32 * i:32 * (i + 1)], "little") for i in range(13))
    return q_int, cts_int


def q() -> int:
    """constant.py:6-7: the BN254 scalar field order."""
    return _params()[0]


def data_block_size() -> int:
    """constant.py:10-11: rows per data commitment."""
    return 128


def cts() -> List[int]:
    """constant.py:14-30: the 13 MiMC7 round constants (a fresh list per call)."""
    return list(_params()[1])
