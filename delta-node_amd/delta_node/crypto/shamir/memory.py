"""Opt-in share-block memory built from physical chunks (dn_block_alloc).

The split writes 330 B per element at 3-of-5 and its rate follows the
physical pages of the share block.  `chunked_block` returns a
uint8 device tensor whose memory is `chunk_bytes` physical chunks
(hipMemCreate) mapped back to back — a composition the caller chooses instead
of one allocation's luck.  Every API keeps accepting tensors from any
allocator; this is only a way to get one.  The tensor owns the block: the
memory is unmapped and released (after a device synchronise) when the last
reference goes.
"""
from __future__ import annotations

import ctypes
from typing import Sequence, Union

from . import _native

__all__ = ["chunked_block", "granularity"]


class _Block:
    """A dn_block_alloc allocation seen through __cuda_array_interface__ (v3):
    torch.as_tensor keeps this object alive as long as the tensor (its
    deleter drops the reference), and __del__ frees the block."""

    def __init__(self, nbytes: int, chunk_bytes: int, device: int, shape):
        self._lib = _native.lib()
        p = ctypes.c_void_p()
        _native.check(self._lib.dn_block_alloc(nbytes, chunk_bytes, device, ctypes.byref(p)))
        self.ptr = p.value
        self.__cuda_array_interface__ = {"shape": tuple(shape), "typestr": "|u1", "data": (self.ptr, False),
                                         "version": 3, "strides": None}

    def __del__(self):
        if getattr(self, "ptr", None):
            self._lib.dn_block_free(self.ptr)
            self.ptr = None


def granularity(device: int = 0) -> int:
    g = ctypes.c_uint64()
    _native.check(_native.lib().dn_block_granularity(device, ctypes.byref(g)))
    return g.value


def chunked_block(shape: Union[int, Sequence[int]], chunk_bytes: int = 2 << 20, device=None):
    """uint8 device tensor of `shape` whose memory is `chunk_bytes` physical
    chunks mapped back to back (0: the library default, 2 MiB)."""
    import math

    import torch

    dev = torch.device(device) if device is not None else _native.require_device()
    if dev.type != "cuda":
        raise ValueError("chunked_block: a HIP device is required")
    idx = dev.index if dev.index is not None else torch.cuda.current_device()
    shape = (int(shape),) if isinstance(shape, int) else tuple(int(s) for s in shape)
    nbytes = max(1, math.prod(shape))
    blk = _Block(nbytes, int(chunk_bytes), idx, shape)
    with torch.cuda.device(idx):
        t = torch.as_tensor(blk, device=dev)
    if t.data_ptr() != blk.ptr or t.dtype != torch.uint8:
        raise RuntimeError("chunked_block: the tensor does not alias the block")
    return t
