"""Share-block memory built from 16 MiB physical chunks (dn_block_alloc).

The split writes 330 B per element at 3-of-5 (70 % of its traffic) and its
rate follows the physical pages of the share block: a 5.5 GB
block from one hipMalloc lands in a fast or a slow class (0.66 / 0.78 of
8 TB/s for the split).  A block built from physical chunks (CHUNK_BYTES)
mapped back to back (hipMemCreate / hipMemMap) ran in the fast class every
time it was measured — 10 of 10 blocks at 0.786-0.800 against 6 of 10 torch.empty blocks
(profiles/r04/a/block_probe.jsonl, and round 1's place_vmm2/3) — so the vector
API allocates the share blocks it returns here (`share_block`), and callers
may too.  Every API keeps accepting tensors from any allocator.

Blocks are pooled: when the last tensor over a block goes, the block returns
to an idle list (keyed by size) and the next request of that size reuses it
without new mappings.  Reuse is stream-ordered, as in torch's caching
allocator: a block remembers the stream it was allocated on (and any stream
`record_stream` adds); when it goes idle an event is recorded on each of them
(dn_block_record), and a request on stream S takes an idle block only when
every such event is on S or has completed (dn_block_acquire) — the caller
owns the shares it was handed (the reference's make_shares returns fresh
objects, shamir.py:62-66), so no other stream's request gets them while that
caller's work on them is still queued.  Only when a new block cannot be
allocated does S wait (on the device, hipStreamWaitEvent) for a busy idle
block instead.  A freed block waits for its own events, not the device.

The pool holds at most `POOL_IDLE_BYTES`, and only while the device keeps
`POOL_MIN_FREE` free beside them; before a new block is mapped, idle blocks
(oldest first) are released until it fits with that headroom.  torch does
not see this memory: `empty_cache()` releases the idle blocks (call it with
torch.cuda.empty_cache()), and it runs by itself when torch reports an
out-of-memory error, so the caller's retry finds the memory free.  Below
`CHUNKED_MIN_BYTES` (data that fits the caches, and where mapping costs more
than it saves) `share_block` is torch.empty.

Chunked blocks are not always fast either (r04q: 2 of 12 at 0.66-0.67 of
8 TB/s for the split, the rest 0.72-0.79), and a block's write rate predicts
its split (5.6-5.7 TB/s -> 0.66-0.67, >= 6.9 TB/s -> >= 0.78;
profiles/r04/q/block_class.jsonl).  So a NEW share block of at least
`PROBE_MIN_BYTES` is probed once (one timed write in the split's order:
per tile, every row's slice) and kept only if it writes
at >= `PROBE_KEEP` of the best rate this process has seen on the device
for blocks of that many rows and that size class (log2 of the bytes);
otherwise up to `PROBE_TRIES` blocks (`PROBE_TRIES_SMALL` under 1 GiB; at
most `PROBE_BUDGET` bytes of them, within the device's free memory) are
mapped and the fastest is kept (the others are freed after the choice, so a
retry cannot get their pages back).  The first block of a class on a device
is the fastest of `PROBE_FIRST` (`PROBE_FIRST_SMALL` under 1 GiB) tries, or
the first to reach `PROBE_FAST`.  A request stops trying once its tries have
taken `PROBE_TIME_BUDGET` seconds (the best block so far is kept).

A freed block's virtual range stays reserved (csrc/vmm_block.cpp,
dn_block_free: a range reused at a freed block's address does not give the
GPU the new mapping).  The retired bytes are counted
(dn_block_retired_bytes); once they would pass `RETIRE_BUDGET`, share blocks
are torch.empty memory (the caching allocator reuses its own ranges) and no
new block is probed, so a long-running process never exhausts the address
space.
"""
from __future__ import annotations

import ctypes
import itertools
import math
import threading
import time
import weakref
from typing import Dict, List, Optional, Sequence, Tuple, Union

from . import _native

__all__ = ["share_block", "chunked_block", "empty_cache", "granularity", "pool_stats", "block_rate",
           "record_stream", "retired_bytes"]

CHUNK_BYTES = 16 << 20         # physical chunk of a pooled block
CHUNKED_MIN_BYTES = 64 << 20   # smaller share blocks: torch.empty
POOL_IDLE_BYTES = 32 << 30     # most idle bytes the pool keeps mapped
POOL_MIN_FREE = 16 << 30       # device bytes kept free beside the idle blocks
PROBE_MIN_BYTES = 64 << 20     # new share blocks from this size up are write-rate probed (every chunked one)
# most blocks mapped for one request (blocks of 1 GiB or more); a request
# stops at the first block close to the best rate, so more tries are spent
# only where the memory handed out is slow: one box's fifth 5.5 GB block was
# the best of 4 slow tries (5.8 TB/s, its split 1.52 ms against 1.26-1.29;
# profiles/r05/final4/)
PROBE_TRIES = 8
# ... for smaller blocks (a try maps a few chunks and writes for microseconds;
# within PROBE_BUDGET): a 2^21 shard's block took the best of 12 slow tries on
# some boxes, 48 found a fast one (bench --log2n 21: 8.58-8.60 vs 8.46-8.49e9
# elements/s, profiles/r05/ac/)
PROBE_TRIES_SMALL = 48
PROBE_KEEP = 0.96              # fraction of the best rate seen that a block must reach
# the first block of a class (no rate to compare with yet): the fastest of this
# many tries — 2 from 1 GiB up (each try maps and writes gigabytes: the cold
# first call), 4 below (a 2^21 shard's first 692 MB block was the best of two
# at 5.7-5.9 TB/s while its later blocks reached 6.2-6.7, profiles/r05/ak/;
# best of 4: the 2^21 line 8.78-8.85 vs 8.76-8.81e9 elements/s, its split
# 0.159-0.162 vs 0.163-0.164 ms, at up to ~70 probes once, profiles/r05/al/)
PROBE_FIRST = 2
PROBE_FIRST_SMALL = 4
PROBE_FAST = 6.8e12            # the first block of a class keeps at once at this tiled-probe rate (B/s)
PROBE_BUDGET = 48 << 30        # most bytes mapped at once for one request's tries (and
                               # never more than the device has free beyond POOL_MIN_FREE)
# most wall time one request spends on its tries AND on freeing the tries it
# rejects (a 5.5 GB block of 16 MiB chunks: ~3-7 ms to map, ~3 ms to probe,
# ~5 ms to free): a request stops trying once the tries so far plus the
# frees they imply (each at the measured cost of a free of that size) pass it,
# so the worst case, every try slow, stays near this instead of PROBE_TRIES
# tries and their frees (bench rows.draw_split.cold.cold_worst_ms)
PROBE_TIME_BUDGET = 0.05
# virtual address space that freed blocks may retire before new share blocks
# come from torch.empty instead (x86-64 user space: 2^47 bytes)
RETIRE_BUDGET = 64 << 40

_lock = threading.RLock()
_idle: Dict[Tuple[int, int, int], List[Tuple[int, int]]] = {}  # (device, nbytes, chunk) -> [(age, ptr)]
_idle_bytes = 0
_age = itertools.count()
_stats = {"allocs": 0, "reuses": 0, "frees": 0, "probed": 0, "rejected": 0, "waits": 0, "busy_skips": 0,
          "trimmed": 0, "record_failures": 0, "free_failures": 0, "budget_stops": 0, "va_fallbacks": 0}
_best_rate: Dict[Tuple[int, int, int], float] = {}  # (device, rows, log2 bytes) -> fastest probed write rate (B/s)
_rates: Dict[int, float] = {}      # block pointer -> its probed write rate
_sizes: Dict[int, int] = {}        # block pointer -> its bytes (dn_block_alloc blocks of this module)
_free_secs: Dict[int, float] = {}  # block bytes -> seconds one dn_block_free of that size took (last measured)
_live: Dict[int, "weakref.ref"] = {}  # block pointer -> its live _Block (record_stream)
_observer = False


def _raw_stream(stream) -> int:
    if stream is None:
        return 0
    return int(getattr(stream, "cuda_stream", stream))


def _free_ptr(ptr: int, streams: Sequence[int] = ()) -> None:
    """Free a block after its uses on `streams` (events recorded here) and the
    ones recorded when it went idle (dn_block_free waits for them)."""
    _rates.pop(ptr, None)
    L = _native.lib()
    for s in streams:
        _native.check(L.dn_block_record(ptr, s or None))
    t0 = time.perf_counter()
    if L.dn_block_free(ptr):
        _stats["free_failures"] += 1
    nbytes = _sizes.pop(ptr, None)
    if nbytes:
        _free_secs[nbytes] = time.perf_counter() - t0
    _stats["frees"] += 1


def retired_bytes() -> int:
    """Virtual address space retired by freed blocks (dn_block_retired_bytes)."""
    b = ctypes.c_uint64()
    _native.check(_native.lib().dn_block_retired_bytes(ctypes.byref(b)))
    return b.value


def _sync_device(index: int) -> None:
    import torch

    torch.cuda.synchronize(index)


def _mem_info(index: int) -> Tuple[int, int]:
    import torch

    return torch.cuda.mem_get_info(index)


class _Block:
    """One dn_block_alloc block seen through __cuda_array_interface__ (v3).
    torch.as_tensor keeps this object alive as long as the tensor; when it
    goes, events are recorded on the streams that used the block and the block
    returns to the idle pool (or is freed: pool full, device short of memory,
    or pooled=False)."""

    def __init__(self, ptr: int, key: Tuple[int, int, int], shape, pooled: bool, stream: int):
        self.ptr, self.key, self.pooled = ptr, key, pooled
        self.streams = {stream}
        self.__cuda_array_interface__ = {"shape": tuple(shape), "typestr": "|u1", "data": (ptr, False),
                                         "version": 3, "strides": None}

    def __del__(self):
        global _idle_bytes
        ptr, self.ptr = getattr(self, "ptr", None), None
        if not ptr:
            return
        try:
            _live.pop(ptr, None)
            L = _native.lib()
            try:
                for s in self.streams:
                    _native.check(L.dn_block_record(ptr, s or None))
            except Exception:
                # an event could not be recorded (a stream destroyed before the
                # tensor, a HIP error): the block's uses are not all tracked, so
                # it is neither pooled nor freed on events — the block's device
                # drains, then the block is freed (and counted)
                _stats["record_failures"] += 1
                _sync_device(self.key[0])
                _free_ptr(ptr)
                return
            if self.pooled:
                nbytes = self.key[1]
                with _lock:
                    if _idle_bytes + nbytes <= POOL_IDLE_BYTES and _mem_info(self.key[0])[0] >= POOL_MIN_FREE:
                        _idle.setdefault(self.key, []).append((next(_age), ptr))
                        _idle_bytes += nbytes
                        return
            _free_ptr(ptr)
        except Exception:  # interpreter shutdown: the process releases the memory
            pass


class _View:
    """A borrowed view of block memory for the probe (frees nothing)."""

    def __init__(self, ptr: int, nbytes: int):
        self.__cuda_array_interface__ = {"shape": (nbytes,), "typestr": "|u1", "data": (ptr, False),
                                         "version": 3, "strides": None}


def _on_oom(*_args) -> None:
    try:
        empty_cache()
    except Exception:
        pass


def _attach_oom_observer() -> None:
    """torch's out-of-memory error releases the idle blocks (torch cannot see them)."""
    global _observer
    if _observer:
        return
    _observer = True
    try:
        import torch

        torch._C._cuda_attach_out_of_memory_observer(_on_oom)
    except Exception:  # an older torch: empty_cache() stays the caller's call
        pass


def _take_idle(key: Tuple[int, int, int], stream: int, wait: bool = False) -> Optional[int]:
    """An idle block of `key` usable on `stream`: one whose recorded uses are
    on `stream` or complete; with wait, any (the stream waits for its events)."""
    global _idle_bytes
    L = _native.lib()
    with _lock:
        lst = _idle.get(key)
        if not lst:
            return None
        for i in range(len(lst) - 1, -1, -1):  # the most recently idled first
            ptr = lst[i][1]
            rc = L.dn_block_acquire(ptr, stream or None, 1 if wait else 0)
            if rc == _native.DN_ERR_RETRY:
                _stats["busy_skips"] += 1
                continue
            _native.check(rc)
            lst.pop(i)
            _idle_bytes -= key[1]
            _stats["reuses"] += 1
            _stats["waits"] += int(wait)
            return ptr
    return None


def _trim_for(nbytes: int, index: int) -> None:
    """Release idle blocks (oldest first) until `nbytes` more fit on the
    device with POOL_MIN_FREE to spare."""
    global _idle_bytes
    with _lock:
        if not _idle_bytes:
            return
        free = _mem_info(index)[0]
        order = sorted((age, key, ptr) for key, lst in _idle.items() if key[0] == index for age, ptr in lst)
        for age, key, ptr in order:
            if free >= nbytes + POOL_MIN_FREE:
                break
            _idle[key].remove((age, ptr))
            if not _idle[key]:
                del _idle[key]
            _idle_bytes -= key[1]
            _free_ptr(ptr)
            _stats["trimmed"] += 1
            free += key[1]


def _alloc_raw(nbytes: int, chunk_bytes: int, index: int) -> int:
    p = ctypes.c_void_p()
    rc = _native.lib().dn_block_alloc(nbytes, int(chunk_bytes), index, ctypes.byref(p))
    if rc:
        empty_cache()  # idle blocks of other sizes may hold the memory
        rc = _native.lib().dn_block_alloc(nbytes, int(chunk_bytes), index, ctypes.byref(p))
    _native.check(rc)
    _stats["allocs"] += 1
    _sizes[p.value] = int(nbytes)
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
    # rates compare within one block class: row count and size (log2 of the bytes)
    kind = (dev.index, int(shape[0]) if len(shape) == 2 else 0, max(1, nbytes).bit_length())
    best = _best_rate.get(kind)
    from . import field

    tiled = len(shape) == 2 and int(shape[0]) > 0 and int(shape[1]) % field.TILE_BYTES == 0
    cands: List[Tuple[float, int]] = []
    most = PROBE_TRIES if nbytes >= (1 << 30) else PROBE_TRIES_SMALL
    first = PROBE_FIRST if nbytes >= (1 << 30) else PROBE_FIRST_SMALL
    spare = max(0, _mem_info(dev.index)[0] - POOL_MIN_FREE)  # torch keeps its margin
    tries = max(1, min(most, PROBE_BUDGET // max(1, nbytes), spare // max(1, nbytes)))
    # every rejected try retires its range: stay within the address-space budget
    tries = max(1, min(tries, (RETIRE_BUDGET - _retired()) // max(1, nbytes)))
    t0 = time.perf_counter()
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
        if best is None and tiled and rate >= PROBE_FAST:  # the class's first block, in the fast class
            break
        if best is None:
            if k >= first - 1:  # the class's first block on this device: the fastest of `first`
                break
        elif rate >= PROBE_KEEP * best:
            break
        if k + 1 < tries:
            # the tries so far, one more, and the frees of all but the kept one
            # (each at the last measured free of this size, else a try's cost)
            spent = time.perf_counter() - t0
            per_try = spent / (k + 1)
            free_cost = _free_secs.get(nbytes, per_try)
            if spent + per_try + (k + 1) * free_cost > PROBE_TIME_BUDGET:
                _stats["budget_stops"] += 1  # out of time for this request: keep the best so far
                break
    rate, keep = max(cands)
    stream = _current_stream(dev.index)  # the probe wrote the rejected blocks on this stream
    for r, p in cands:
        if p != keep:
            _free_ptr(p, (stream,))
            _stats["rejected"] += 1
    _best_rate[kind] = max([best or 0.0] + [r for r, _ in cands])
    _rates[keep] = rate
    return keep


def _retired() -> int:
    return retired_bytes()


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


def _current_stream(index: int) -> int:
    import torch

    return int(torch._C._cuda_getCurrentRawStream(index))


def chunked_block(shape: Union[int, Sequence[int]], chunk_bytes: int = CHUNK_BYTES, device=None,
                  pooled: bool = True, probe: bool = False):
    """uint8 device tensor of `shape` whose memory is `chunk_bytes` physical
    chunks mapped back to back (from the idle pool when one of this size is
    free for the current stream; probe: a new block is write-rate probed, see
    the module docstring).  The block is recorded as used on the current
    stream; `record_stream` adds others."""
    import torch

    dev = _device_index(device)
    shape = (int(shape),) if isinstance(shape, int) else tuple(int(s) for s in shape)
    nbytes = max(1, math.prod(shape))
    key = (dev.index, nbytes, int(chunk_bytes))
    stream = _current_stream(dev.index)
    _attach_oom_observer()
    ptr = _take_idle(key, stream)
    if ptr is None:
        _trim_for(nbytes, dev.index)
        try:
            if probe and nbytes >= PROBE_MIN_BYTES:
                ptr = _alloc_probed(nbytes, chunk_bytes, dev, shape)
            else:
                ptr = _alloc_raw(nbytes, chunk_bytes, dev.index)
        except RuntimeError:
            ptr = _take_idle(key, stream, wait=True)  # out of memory: order after a busy idle block's users
            if ptr is None:
                raise
    blk = _Block(ptr, key, shape, pooled, stream)
    if dev.index == torch.cuda.current_device():  # (a device switch costs two hipSetDevice per call)
        t = torch.as_tensor(blk, device=dev)
    else:
        with torch.cuda.device(dev.index):
            t = torch.as_tensor(blk, device=dev)
    if t.data_ptr() != ptr or t.dtype != torch.uint8 or tuple(t.shape) != shape:
        raise RuntimeError("chunked_block: the tensor does not alias the block")
    _live[ptr] = weakref.ref(blk)
    return t


def record_stream(t, stream) -> None:
    """Mark the pooled block under tensor `t` as used on `stream` (a
    torch.cuda.Stream or a raw handle): when the block goes idle, requests on
    other streams wait for the work queued on `stream` until then.  torch's
    own Tensor.record_stream does nothing for memory torch did not allocate.
    A tensor that is not over a pooled block is left alone."""
    p = t.data_ptr()
    for base, ref in list(_live.items()):
        blk = ref()
        if blk is not None and base <= p < base + blk.key[1]:
            blk.streams.add(_raw_stream(stream))
            return


def share_block(shape: Union[int, Sequence[int]], device=None):
    """A share block (uint8 [n_shares, vec_bytes(n)] or any shape): pooled
    chunked memory (CHUNK_BYTES) from CHUNKED_MIN_BYTES up, torch.empty below."""
    import torch

    dev = _device_index(device)
    shape = (int(shape),) if isinstance(shape, int) else tuple(int(s) for s in shape)
    nbytes = math.prod(shape)
    if nbytes < CHUNKED_MIN_BYTES:
        return torch.empty(shape, dtype=torch.uint8, device=dev)
    if not _has_idle((dev.index, nbytes, CHUNK_BYTES)) and _retired() + nbytes > RETIRE_BUDGET:
        _stats["va_fallbacks"] += 1  # address space retired past the budget: no new mappings
        return torch.empty(shape, dtype=torch.uint8, device=dev)
    return chunked_block(shape, CHUNK_BYTES, dev, probe=True)


def _has_idle(key) -> bool:
    with _lock:
        return bool(_idle.get(key))


def empty_cache() -> None:
    """Release every idle pooled block (their memory returns to the device,
    each after the work recorded on it)."""
    global _idle_bytes
    with _lock:
        ptrs = [p for lst in _idle.values() for _, p in lst]
        _idle.clear()
        _idle_bytes = 0
    for p in ptrs:
        _free_ptr(p)


def pool_stats() -> dict:
    with _lock:
        stats = {**_stats, "idle_blocks": sum(len(v) for v in _idle.values()), "idle_bytes": _idle_bytes}
    try:
        stats["retired_bytes"] = retired_bytes()
    except Exception:  # a scripted library without the counter
        stats["retired_bytes"] = None
    return stats
