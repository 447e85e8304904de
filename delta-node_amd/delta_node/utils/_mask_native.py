"""ctypes binding of the mask-PRG C-ABI (include/dn_mask.h) in libdn_shamir.so."""
from __future__ import annotations

import ctypes
from typing import List, Optional, Sequence, Union

from ..crypto.shamir import _native

MAX_GENS = 16
EXPORTS = ("dn_pcg64_seed", "dn_pcg64_advance", "dn_bounded_i64_accumulate", "dn_bounded_i64_rejects",
           "dn_unfix_precision", "dn_i64_sum")


class PCG64(ctypes.Structure):
    """Mirror of dn_pcg64_t (numpy PCG64 state: 128-bit state and increment)."""

    _fields_ = [("state_hi", ctypes.c_uint64), ("state_lo", ctypes.c_uint64),
                ("inc_hi", ctypes.c_uint64), ("inc_lo", ctypes.c_uint64)]

    @property
    def state(self) -> int:
        return (self.state_hi << 64) | self.state_lo

    @property
    def inc(self) -> int:
        return (self.inc_hi << 64) | self.inc_lo


def lib() -> ctypes.CDLL:
    L = _native.lib()
    if not getattr(L, "_dn_mask_bound", False):  # argtypes, once per loaded library
        vp, u64, i32, i64 = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int, ctypes.c_int64
        L.dn_pcg64_seed.restype = i32
        L.dn_pcg64_seed.argtypes = [ctypes.POINTER(ctypes.c_uint32), i32, ctypes.POINTER(PCG64)]
        L.dn_pcg64_advance.restype = i32
        L.dn_pcg64_advance.argtypes = [ctypes.POINTER(PCG64), u64]
        L.dn_bounded_i64_accumulate.restype = i32
        L.dn_bounded_i64_accumulate.argtypes = [ctypes.POINTER(PCG64), ctypes.POINTER(ctypes.c_int32),
                                                ctypes.POINTER(ctypes.c_uint64), i32, i64, u64, vp, vp, i32, vp,
                                                u64, u64, vp, vp]
        L.dn_bounded_i64_rejects.restype = i32
        L.dn_bounded_i64_rejects.argtypes = [ctypes.POINTER(PCG64), u64, u64, u64, vp, vp, ctypes.c_uint32, vp]
        L.dn_i64_sum.restype = i32
        L.dn_i64_sum.argtypes = [ctypes.POINTER(vp), i32, vp, u64, vp]
        L.dn_unfix_precision.restype = i32
        L.dn_unfix_precision.argtypes = [vp, vp, u64, i32, vp]
        L._dn_mask_bound = True
    return L


def entropy_words(seed: Union[int, bytes, Sequence[int]]) -> List[int]:
    """numpy SeedSequence entropy -> uint32 words (one per byte of a bytes
    seed, the little-endian 32-bit words of an int)."""
    def int_words(v: int) -> List[int]:
        if v < 0:
            raise ValueError("expected non-negative integer")
        if v == 0:
            return [0]
        out = []
        while v:
            out.append(v & 0xFFFFFFFF)
            v >>= 32
        return out

    if isinstance(seed, int):
        return int_words(seed)
    if isinstance(seed, (bytes, bytearray)):  # one word per byte (every byte < 2^32)
        return list(seed)
    words: List[int] = []
    for v in (list(seed) if isinstance(seed, (bytes, bytearray)) else seed):
        words.extend(int_words(int(v)))
    return words


def pcg64(seed) -> PCG64:
    """numpy PCG64(SeedSequence(seed)) state (host)."""
    w = entropy_words(seed)
    arr = (ctypes.c_uint32 * max(1, len(w)))(*w)
    g = PCG64()
    _native.check(lib().dn_pcg64_seed(arr, len(w), ctypes.byref(g)))
    return g


def advance(g: PCG64, delta: int) -> PCG64:
    h = PCG64(g.state_hi, g.state_lo, g.inc_hi, g.inc_lo)
    _native.check(lib().dn_pcg64_advance(ctypes.byref(h), delta))
    return h


def accumulate(gens: Sequence[PCG64], signs: Sequence[int], out, n: int, low: int, rng: int, *, base_i64=None,
               base_f64=None, precision: int = 0, raw_offsets: Optional[Sequence[int]] = None,
               elem_begin: int = 0, elem_end: Optional[int] = None, rejects=None) -> None:
    k = len(gens)
    G = (PCG64 * max(1, k))(*gens)
    S = (ctypes.c_int32 * max(1, k))(*signs)
    R = (ctypes.c_uint64 * max(1, k))(*(raw_offsets or [0] * k))
    _native.check(lib().dn_bounded_i64_accumulate(
        G, S, R, k, low, rng, _native._ptr(base_i64), _native._ptr(base_f64), precision, out.data_ptr(),
        elem_begin, n if elem_end is None else elem_end, _native._ptr(rejects), _native.stream_ptr()))


def list_rejects(g: PCG64, rng: int, raw_begin: int, raw_end: int, capacity: int, dev):
    import torch

    idx = torch.zeros(max(1, capacity), dtype=torch.int64, device=dev)
    cnt = torch.zeros(1, dtype=torch.int32, device=dev)
    _native.check(lib().dn_bounded_i64_rejects(ctypes.byref(g), rng, raw_begin, raw_end, idx.data_ptr(),
                                               cnt.data_ptr(), capacity, _native.stream_ptr()))
    c = int(cnt.item())
    return c, sorted(int(v) for v in idx[: min(c, capacity)].cpu().tolist())


def i64_sum(inputs, out, n: int) -> None:
    ptrs = (ctypes.c_void_p * len(inputs))(*[t.data_ptr() for t in inputs])
    _native.check(lib().dn_i64_sum(ptrs, len(inputs), out.data_ptr(), n, _native.stream_ptr()))


def unfix(inp, out, n: int, precision: int) -> None:
    _native.check(lib().dn_unfix_precision(inp.data_ptr(), out.data_ptr(), n, precision, _native.stream_ptr()))
