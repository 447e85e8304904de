"""Share-block memory built from 2 MiB physical chunks (dn_block_alloc).

The split writes 330 B per element at 3-of-5 (70 % of its traffic) and its
rate follows the physical pages of the share block: a 5.5 GB
block from one hipMalloc lands in a fast or a slow class (0.66 / 0.78 of
8 TB/s for the split).  A block built from 2 MiB physical chunks mapped back to
back (hipMemCreate / hipMemMap) ran in the fast class every time it was
measured — 10 of 10 blocks at 0.786-0.800 against 6 of 10 torch.empty blocks
(profiles/r04/a/block_probe.jsonl, and round 1's place_vmm2/3) — so the vector
API allocates the share blocks it returns here (`share_block`), and callers
may too.  Every API keeps accepting tensors from any allocator.

Blocks are pooled: when the last tensor over a block goes, the block returns
to an idle list (keyed by size, at most `POOL_IDLE_BYTES` held) and the next
request of that size reuses it without new mappings; `empty_cache()` releases
the idle blocks.  Below `CHUNKED_MIN_BYTES` (data that fits the caches, and
where mapping costs more than it saves) `share_block` is torch.empty.

Chunked blocks are not always fast either (r04q: 2 of 12 at 0.66-0.67 of
8 TB/s for the split, the rest 0.72-0.79), and a block's write rate predicts
its split (5.6-5.7 TB/s -> 0.66-0.67, >= 6.9 TB/s -> >= 0.78;
profiles/r04/q/block_class.jsonl).  So a NEW share block of at least
`PROBE_MIN_BYTES` is probed once (one timed write in the split's order:
per tile, every row's slice) and kept only if it writes
at >= `PROBE_KEEP` of the best rate this process has seen on the device
for blocks of that many rows;
otherwise up to `PROBE_TRIES` blocks (at most `PROBE_BUDGET` bytes of them)
are mapped and the fastest is kept (the others are freed after the choice, so
a retry cannot get their pages back).
The first large block on a device is the faster of two.
"""
from __future__ import annotations

import ctypes
import math
import threading
from typing import Dict, List, Optional, Sequence, Tuple, Union

from . import _native

__all__ = ["share_block", "chunked_block", "empty_cache", "granularity", "pool_stats", "block_rate"]

CHUNK_BYTES = 2 << 20          # physical chunk of a pooled block
CHUNKED_MIN_BYTES = 64 << 20   # smaller share blocks: torch.empty
POOL_IDLE_BYTES = 64 << 30     # most idle bytes the pool keeps mapped
PROBE_MIN_BYTES = 256 << 20    # new share blocks from this size up are write-rate probed
PROBE_TRIES = 4                # most blocks mapped for one request
PROBE_KEEP = 0.96              # fraction of the best rate seen that a block must reach
PROBE_BUDGET = 24 << 30        # most bytes mapped at once for one request's tries

_lock = threading.Lock()
_idle: Dict[Tuple[int, int, int], List[int]] = {}  # (device, nbytes, chunk) -> idle block pointers
_idle_bytes = 0
_stats = {"allocs": 0, "reuses": 0, "frees": 0, "probed": 0, "rejected": 0}
_best_rate: Dict[Tuple[int, int], float] = {}  # (device, rows) -> fastest probed write rate (bytes/s)
_rates: Dict[int, float] = {}      # block pointer -> its probed write rate


def _free_ptr(ptr: int) -> None:
    _rates.pop(ptr, None)
    _native.lib().dn_block_free(ptr)
    _stats["frees"] += 1


class _Block:
    """One dn_block_alloc block seen through __cuda_array_interface__ (v3).
    torch.as_tensor keeps this object alive as long as the tensor; when it
    goes, the block returns to the idle pool (or is freed: pool full, or
    pooled=False)."""

    def __init__(self, ptr: int, key: Tuple[int, int, int], shape, pooled: bool):
        self.ptr, self.key, self.pooled = ptr, key, pooled
        self.__cuda_array_interface__ = {"shape": tuple(shape), "typestr": "|u1", "data": (ptr, False),
                                         "version": 3, "strides": None}

    def __del__(self):
        global _idle_bytes
        ptr, self.ptr = getattr(self, "ptr", None), None
        if not ptr:
            return
        try:
            if self.pooled:
                with _lock:
                    if _idle_bytes + self.key[1] <= POOL_IDLE_BYTES:
                        _idle.setdefault(self.key, []).append(ptr)
                        _idle_bytes += self.key[1]
                        return
            _free_ptr(ptr)
        except Exception:  # interpreter shutdown: the process releases the memory
            pass


class _View:
    """A borrowed view of block memory for the probe (frees nothing)."""

    def __init__(self, ptr: int, nbytes: int):
        self.__cuda_array_interface__ = {"shape": (nbytes,), "typestr": "|u1", "data": (ptr, False),
                                         "version": 3, "strides": None}


def _alloc_raw(nbytes: int, chunk_bytes: int, index: int) -> int:
    p = ctypes.c_void_p()
    rc = _native.lib().dn_block_alloc(nbytes, int(chunk_bytes), index, ctypes.byref(p))
    if rc:
        empty_cache()  # idle blocks of other sizes may hold the memory
        rc = _native.lib().dn_block_alloc(nbytes, int(chunk_bytes), index, ctypes.byref(p))
    _native.check(rc)
    _stats["allocs"] += 1
    return p.value


def _write_rate(ptr: int, nbytes: int, dev, shape) -> float:
    """Bytes/s of writing the block (best of two, after a first touch): for a
    block of rows of whole tiles (a share or coefficient block) in the order
    a split writes it (dn_block_probe_rows: per tile, every row's slice) —
    a linear fill ran at the same rate on blocks whose split differed by
    20 % (profiles/r04/x/ vs r04/y/); else one linear fill."""
    import torch

    from . import field

    rows = int(shape[0]) if len(shape) == 2 else 0
    tiled = rows > 0 and int(shape[1]) % field.TILE_BYTES == 0
    with torch.cuda.device(dev.index):
        t = torch.as_tensor(_View(ptr, nbytes), device=dev)
        stream = torch.cuda.current_stream()

        def write():
            if tiled:
                _native.check(_native.lib().dn_block_probe_rows(ptr, rows, int(shape[1]), stream.cuda_stream))
            else:
                t.fill_(0)

        write()
        best = None
        for _ in range(2):
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record(stream)
            write()
            e.record(stream)
            e.synchronize()
            ms = s.elapsed_time(e)
            best = ms if best is None else min(best, ms)
        del t
    return (rows * int(shape[1]) if tiled else nbytes) / (best * 1e-3)


def _alloc_probed(nbytes: int, chunk_bytes: int, dev, shape) -> int:
    """A new block, write-rate probed (see the module docstring)."""
    kind = (dev.index, int(shape[0]) if len(shape) == 2 else 0)  # rates compare within one block shape class
    best = _best_rate.get(kind)
    cands: List[Tuple[float, int]] = []
    tries = max(1, min(PROBE_TRIES, PROBE_BUDGET // max(1, nbytes)))
    for k in range(tries):
        try:
            ptr = _alloc_raw(nbytes, chunk_bytes, dev.index)
        except RuntimeError:
            if cands:  # out of memory for another try: keep the best so far
                break
            raise
        rate = _write_rate(ptr, nbytes, dev, shape)
        _stats["probed"] += 1
        cands.append((rate, ptr))
        if best is None:
            if k >= 1:  # the first large block on this device: the faster of two
                break
        elif rate >= PROBE_KEEP * best:
            break
    rate, keep = max(cands)
    for r, p in cands:
        if p != keep:
            _free_ptr(p)
            _stats["rejected"] += 1
    _best_rate[kind] = max([best or 0.0] + [r for r, _ in cands])
    _rates[keep] = rate
    return keep


def block_rate(t) -> Optional[float]:
    """The probed write rate (bytes/s) of the block `t` starts at, if it was probed."""
    return _rates.get(t.data_ptr())


def granularity(device: int = 0) -> int:
    g = ctypes.c_uint64()
    _native.check(_native.lib().dn_block_granularity(device, ctypes.byref(g)))
    return g.value


def _device_index(device):
    import torch

    dev = torch.device(device) if device is not None else _native.require_device()
    if dev.type != "cuda":
        raise ValueError("share blocks live on a HIP device")
    return torch.device("cuda", dev.index if dev.index is not None else torch.cuda.current_device())


def chunked_block(shape: Union[int, Sequence[int]], chunk_bytes: int = CHUNK_BYTES, device=None,
                  pooled: bool = True, probe: bool = False):
    """uint8 device tensor of `shape` whose memory is `chunk_bytes` physical
    chunks mapped back to back (from the idle pool when one of this size is
    there; probe: a new block is write-rate probed, see the module docstring)."""
    global _idle_bytes
    import torch

    dev = _device_index(device)
    shape = (int(shape),) if isinstance(shape, int) else tuple(int(s) for s in shape)
    nbytes = max(1, math.prod(shape))
    key = (dev.index, nbytes, int(chunk_bytes))
    ptr = None
    with _lock:
        lst = _idle.get(key)
        if lst:
            ptr = lst.pop()
            _idle_bytes -= nbytes
            _stats["reuses"] += 1
    if ptr is None:
        if probe and nbytes >= PROBE_MIN_BYTES:
            ptr = _alloc_probed(nbytes, chunk_bytes, dev, shape)
        else:
            ptr = _alloc_raw(nbytes, chunk_bytes, dev.index)
    blk = _Block(ptr, key, shape, pooled)
    with torch.cuda.device(dev.index):
        t = torch.as_tensor(blk, device=dev)
    if t.data_ptr() != ptr or t.dtype != torch.uint8 or tuple(t.shape) != shape:
        raise RuntimeError("chunked_block: the tensor does not alias the block")
    return t


def share_block(shape: Union[int, Sequence[int]], device=None):
    """A share block (uint8 [n_shares, vec_bytes(n)] or any shape): pooled
    2 MiB-chunk memory from CHUNKED_MIN_BYTES up, torch.empty below."""
    import torch

    dev = _device_index(device)
    shape = (int(shape),) if isinstance(shape, int) else tuple(int(s) for s in shape)
    if math.prod(shape) < CHUNKED_MIN_BYTES:
        return torch.empty(shape, dtype=torch.uint8, device=dev)
    return chunked_block(shape, CHUNK_BYTES, dev, probe=True)


def empty_cache() -> None:
    """Release every idle pooled block (their memory returns to the device)."""
    global _idle_bytes
    with _lock:
        ptrs = [p for lst in _idle.values() for p in lst]
        _idle.clear()
        _idle_bytes = 0
    for p in ptrs:
        _free_ptr(p)


def pool_stats() -> dict:
    with _lock:
        return {**_stats, "idle_blocks": sum(len(v) for v in _idle.values()), "idle_bytes": _idle_bytes}
