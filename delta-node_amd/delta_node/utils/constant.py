"""BN254 / MiMC7 field parameters (reference: delta_node/utils/constant.py:1-30).

Same names and values: q(), data_block_size(), cts().  Plain Python literals,
usable without the native library as in the reference; the library's copy
(dn_mimc7_params, defined once in csrc/mimc7_consts.hpp for the kernels and
the host chain) is checked equal to these by tests/test_mimc7.py.
"""
from __future__ import annotations

from typing import List

__all__ = ["q", "data_block_size", "cts"]

_Q = 0x30644e72e131a029b85045b68181585d2833e84879b9709143e1f593f0000001
_CTS = (
    0x0,
    0x2e2ebbb178296b63d88ec198f0976ad98bc1d4eb0d921ddd2eb86cb7e70a98e5,
    0x21bfc154b5b071d22d06105663553801f858c1f231020b4c291a729d6281d349,
    0x126cfa352b0e2701442b36e0c2fc88287cfd3bfecce842afc0e3e78d8edb4ad8,
    0x309d7067ab65de1a99fe23f458d0bc3f18c59b6642ef48afc679ef17cb6928c,
    0x194c4693409966960be88513cfe32987c125f71398a782e44973fb8af4798bd8,
    0x5a849684bc58cc0d6e9f319b4dae26db171733bf60f31d978e41d09a75a6319,
    0x18bd4dae5134538bd2f90d41bbb1e330b2a8286ba4a09aca3fbbdcf932534be5,
    0x736c60cd39fd1649d4845b4f9a6ec9baca89fb2de0a3d7eeabe43504b5607fa,
    0x25a6971a9d2c1de9f374378d8f61492b1bd3c46584c076a76c43c3cd1a747512,
    0xa3373d15fa6dce221f83226c02d41f8aea5cfc6da4c9f4981ada1bd4b50f56e,
    0x2b70028e2bf4e008e22eddb78d4190d73c289dc6445b3f64e15f8bd0ec02c672,
    0xb24ef461a71eed93dd366342f9ca4eebb749c8a5a6057c801d538c7c0666ba4,
)


def q() -> int:
    """constant.py:6-7: the BN254 scalar field order."""
    return _Q


def data_block_size() -> int:
    """constant.py:10-11: rows per data commitment."""
    return 128


def cts() -> List[int]:
    """constant.py:14-30: the 13 MiMC7 round constants (a fresh list per call)."""
    return list(_CTS)
