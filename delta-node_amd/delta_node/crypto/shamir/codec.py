"""Share wire codec over whole vectors.

Record e of an encoded share vector is exactly the reference's
`_share_to_bytes((x, y_e))` (shamir.py:28-33): `[len(xb)][xb][yb]` with
minimal big-endian xb / yb.  Records are packed back to back in one uint8
device tensor with int64 offsets[n + 1] (record e = packed[offsets[e]:offsets[e+1]]),
which is what goes to the HTTP peer for receiver x instead of n Python
`bytes` objects.  Encoding / decoding run on the GPU (dn_m521_encode_shares /
dn_m521_decode_shares); `records_to_list` turns a host copy into the
reference's List[bytes] when a caller needs it.
"""
from __future__ import annotations

import ctypes
from typing import List, Tuple

from . import _native, field

EXPORTS = ("dn_m521_codec_scratch_bytes", "dn_m521_encoded_capacity", "dn_m521_encode_shares",
           "dn_m521_decode_shares")
def _lib():
    L = _native.lib()
    if not getattr(L, "_dn_codec_bound", False):  # argtypes, once per loaded library
        vp, u64, i32 = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int
        L.dn_m521_codec_scratch_bytes.restype = u64
        L.dn_m521_codec_scratch_bytes.argtypes = [u64]
        L.dn_m521_encoded_capacity.restype = u64
        L.dn_m521_encoded_capacity.argtypes = [u64, u64]
        L.dn_m521_encode_shares.restype = i32
        L.dn_m521_encode_shares.argtypes = [vp, u64, u64, vp, vp, u64, vp, u64, vp]
        L.dn_m521_decode_shares.restype = i32
        L.dn_m521_decode_shares.argtypes = [vp, u64, vp, u64, vp, vp, vp, vp]
        L._dn_codec_bound = True
    return L


def encode_share_vec(vec, n: int, x: int, *, trim: bool = True):
    """Share x of n elements (uint8 device tensor, tiled) -> (packed uint8, offsets int64[n+1])."""
    import torch

    if not 0 <= x < (1 << 64):
        raise NotImplementedError("encode_share_vec: x must fit 64 bits")
    L = _lib()
    dev = vec.device
    cap = int(L.dn_m521_encoded_capacity(n, x))
    out = torch.empty(max(cap, 1), dtype=torch.uint8, device=dev)
    # every entry is written by the encoder (offsets[n] by the last element)
    offsets = torch.empty(n + 1, dtype=torch.int64, device=dev) if n else torch.zeros(1, dtype=torch.int64, device=dev)
    sb = int(L.dn_m521_codec_scratch_bytes(n))
    scratch = torch.empty(max(sb, 1), dtype=torch.uint8, device=dev)
    _native.check(L.dn_m521_encode_shares(vec.data_ptr(), n, x, offsets.data_ptr(), out.data_ptr(), cap,
                                          scratch.data_ptr(), sb, _native.stream_ptr()))
    if trim:
        out = out[: int(offsets[n].item())]
    return out, offsets


def decode_share_vec(packed, offsets, n: int):
    """(packed, offsets[n+1]) -> (tiled uint8 vector of y mod p, uint64 xs as int64 tensor)."""
    import torch

    L = _lib()
    dev = packed.device
    vec = torch.empty(field.vec_bytes(n), dtype=torch.uint8, device=dev)
    xs = torch.empty(max(n, 1), dtype=torch.int64, device=dev)
    bad = torch.zeros(1, dtype=torch.int32, device=dev)
    _native.check(L.dn_m521_decode_shares(packed.data_ptr(), packed.numel(), offsets.data_ptr(), n, vec.data_ptr(), xs.data_ptr(),
                                          bad.data_ptr(), _native.stream_ptr()))
    nbad = int(bad.item())
    if nbad:
        raise ValueError(f"decode_share_vec: {nbad} records with x > 8 bytes or y > 68 bytes")
    return vec, xs[:n]


def records_to_list(packed_host, offsets_host) -> List[bytes]:
    """Host copy -> the reference's List[bytes] (one record per element)."""
    buf = bytes(packed_host.numpy() if hasattr(packed_host, "numpy") else packed_host)
    off = offsets_host.tolist()
    return [buf[off[i]:off[i + 1]] for i in range(len(off) - 1)]
