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


_scratch_cache = {}  # (device index, stream) -> uint8 scratch tensor (grown on demand)


def _scratch(dev, nbytes: int):
    """Encoder scratch, cached per device and stream (the kernels of one stream
    run in order, so one buffer serves every call queued on it)."""
    import torch

    key = (dev.index, _native.stream_ptr())
    buf = _scratch_cache.get(key)
    if buf is None or buf.numel() < nbytes:
        buf = torch.empty(max(nbytes, 1), dtype=torch.uint8, device=dev)
        _scratch_cache[key] = buf
    return buf


def _out(t, numel: int, dtype, dev, what: str):
    import torch

    if t is None:
        return torch.empty(numel, dtype=dtype, device=dev)
    if not (isinstance(t, torch.Tensor) and t.dtype == dtype and t.device == dev and t.is_contiguous()
            and t.numel() >= numel):
        raise ValueError(f"{what}: expected a contiguous {dtype} tensor of >= {numel} elements on {dev}")
    return t


def encode_share_vec(vec, n: int, x: int, *, trim: bool = True, out=None, offsets=None):
    """Share x of n elements (uint8 device tensor, tiled) -> (packed uint8, offsets int64[n+1]).
    out / offsets: caller buffers (>= encoded_capacity(n, x) bytes, >= n + 1 entries), else allocated.
    trim=True cuts `packed` to its length (one read-back of offsets[n])."""
    import torch

    if not 0 <= x < (1 << 64):
        raise NotImplementedError("encode_share_vec: x must fit 64 bits")
    L = _lib()
    dev = vec.device
    cap = int(L.dn_m521_encoded_capacity(n, x))
    out = _out(out, max(cap, 1), torch.uint8, dev, "encode_share_vec out")
    # every entry is written by the encoder (offsets[n] by the last element)
    if n:
        offsets = _out(offsets, n + 1, torch.int64, dev, "encode_share_vec offsets")[: n + 1]
    else:
        offsets = _out(offsets, 1, torch.int64, dev, "encode_share_vec offsets")[:1]
        offsets.zero_()
    sb = int(L.dn_m521_codec_scratch_bytes(n))
    scratch = _scratch(dev, sb)
    _native.check(L.dn_m521_encode_shares(vec.data_ptr(), n, x, offsets.data_ptr(), out.data_ptr(), cap,
                                          scratch.data_ptr(), sb, _native.stream_ptr()))
    if trim:
        out = out[: int(offsets[n].item())]
    return out, offsets


def encoded_capacity(n: int, x: int) -> int:
    """Bytes the encoder may write for n records of share x (an `out` buffer's size)."""
    return int(_lib().dn_m521_encoded_capacity(n, x))


_flags = {}  # (device index, stream) -> int32 bad-record counter of the checked form


def decode_share_vec(packed, offsets, n: int, *, out=None, xs=None, bad=None):
    """(packed, offsets[n+1]) -> (tiled uint8 vector of y mod p, uint64 xs as int64 tensor).

    out / xs: caller buffers (>= vec_bytes(n) bytes, >= n entries), else allocated.
    bad=None: the call checks for records it cannot represent (x > 8 bytes,
    y > 68 bytes) with one read-back and raises ValueError.  bad=<int32 device
    tensor>: the count of such records is ADDED to it on the device and the
    call does not synchronise — the caller checks it once, at its next sync
    (`check_bad(bad)`), over any number of decodes."""
    import torch

    L = _lib()
    dev = packed.device
    vec = _out(out, field.vec_bytes(n), torch.uint8, dev, "decode_share_vec out")
    xs = _out(xs, max(n, 1), torch.int64, dev, "decode_share_vec xs")
    checked = bad is None
    if checked:
        key = (dev.index, _native.stream_ptr())
        bad = _flags.get(key)
        if bad is None:
            bad = _flags[key] = torch.zeros(1, dtype=torch.int32, device=dev)
        else:
            bad.zero_()
    elif not (isinstance(bad, torch.Tensor) and bad.dtype == torch.int32 and bad.device == dev):
        raise ValueError("decode_share_vec: bad must be an int32 tensor on the packed records' device")
    _native.check(L.dn_m521_decode_shares(packed.data_ptr(), packed.numel(), offsets.data_ptr(), n, vec.data_ptr(),
                                          xs.data_ptr(), bad.data_ptr(), _native.stream_ptr()))
    if checked:
        check_bad(bad)
    return vec, xs[:n]


def check_bad(bad) -> None:
    """Raise if a deferred decode (decode_share_vec(..., bad=flag)) met records
    it cannot represent (one read-back)."""
    nbad = int(bad.item())
    if nbad:
        raise ValueError(f"decode_share_vec: {nbad} records with x > 8 bytes or y > 68 bytes")


def records_to_list(packed_host, offsets_host) -> List[bytes]:
    """Host copy -> the reference's List[bytes] (one record per element)."""
    buf = bytes(packed_host.numpy() if hasattr(packed_host, "numpy") else packed_host)
    off = offsets_host.tolist()
    return [buf[off[i]:off[i + 1]] for i in range(len(off) - 1)]
