"""Share-block memory (delta_node.crypto.shamir.memory, csrc/vmm_block.cpp):
blocks of 16 MiB physical chunks, pooled, aliased by torch tensors through
__cuda_array_interface__; the vector API's default output allocation.  The
split written into a chunked block equals the split into torch.empty memory
byte for byte (the reference's shamir.py:55-66 per element)."""
import gc

import pytest
import torch

from delta_node.crypto import shamir
from delta_node.crypto.shamir import _native, field, memory

pytestmark = pytest.mark.gpu


def dev():
    return torch.device("cuda", 0)


def test_chunked_block_aliases_and_pools():
    memory.empty_cache()
    s0 = memory.pool_stats()
    shape = (5, field.vec_bytes(1 << 18))
    t = memory.chunked_block(shape, device=dev())
    assert t.dtype == torch.uint8 and tuple(t.shape) == shape and t.is_cuda and t.is_contiguous()
    t.fill_(7)
    assert int(t[4, -1].item()) == 7 and int(t.sum(dtype=torch.int64).item()) == 7 * t.numel()
    ptr = t.data_ptr()
    del t
    gc.collect()
    assert memory.pool_stats()["idle_blocks"] == s0["idle_blocks"] + 1
    u = memory.chunked_block(shape, device=dev())  # the idle block of this size comes back
    assert u.data_ptr() == ptr and memory.pool_stats()["reuses"] == s0["reuses"] + 1
    v = u[1:3].clone()  # views and copies behave as device memory
    assert torch.equal(v, u[1:3])
    del u, v
    gc.collect()
    memory.empty_cache()
    st = memory.pool_stats()
    assert st["idle_blocks"] == 0 and st["idle_bytes"] == 0


@pytest.mark.parametrize("chunk", [2 << 20, 64 << 20])
def test_split_into_chunked_block_equals_torch_empty(chunk):
    N, t, n = (1 << 20) + 77, 3, 5
    sec = torch.randint(-(1 << 62), 1 << 62, (N,), dtype=torch.int64, device=dev())
    ss = shamir.SecretShare(t)
    ss.random.seed(3)
    co = ss.draw_coeffs_vec(N, dev())
    vb = field.vec_bytes(N)
    a = torch.empty((n, vb), dtype=torch.uint8, device=dev())
    b = memory.chunked_block((n, vb), chunk, dev())
    a.zero_()
    b.zero_()  # the lanes past N of the last tile are never written
    _native.split_u64(sec, co, a, N, t, n)
    _native.split_u64(sec, co, b, N, t, n)
    assert torch.equal(a, b)
    rec = ss.resolve_shares_vec([b[0], b[2], b[4]], [1, 3, 5], N)
    assert torch.equal(rec, sec)


def test_make_shares_vec_default_output_is_share_block():
    N = 1 << 18  # 5 x vec_bytes = 87 MB >= CHUNKED_MIN_BYTES
    assert 5 * field.vec_bytes(N) >= memory.CHUNKED_MIN_BYTES
    sec = torch.randint(-(1 << 62), 1 << 62, (N,), dtype=torch.int64, device=dev())
    a, b = shamir.SecretShare(3), shamir.SecretShare(3)
    a.random.seed(11)
    b.random.seed(11)
    s0 = memory.pool_stats()
    out = a.make_shares_vec(sec, 5)
    st = memory.pool_stats()
    kept = lambda x: x["allocs"] - x["rejected"] + x["reuses"]  # noqa: E731  (probed tries that were freed excluded)
    assert kept(st) == kept(s0) + 1
    want = torch.empty_like(out)
    b.make_shares_vec(sec, 5, out=want)
    assert torch.equal(out, want) and a.random.getstate() == b.random.getstate()
    small = a.make_shares_vec(sec[:1000], 5)  # below the threshold: torch.empty
    assert kept(memory.pool_stats()) == kept(st)
    assert tuple(small.shape) == (5, field.vec_bytes(1000))


def test_freed_block_address_is_never_reused():
    """A freed block's virtual range is retired (csrc/vmm_block.cpp): the next
    block lands elsewhere, its bytes stay put under later allocations, and the
    torch segments allocated after the free keep theirs (no allocation gets a
    freed block's pages under a live translation).  The cause, reproduced
    without torch by tools/vmm_reuse_probe (modes 5/6, profiles/r05/vmm_reuse/):
    a block mapped with fresh handles at a freed block's address is not the
    memory the GPU accesses there — every word reads back wrong."""
    memory.empty_cache()
    shape = (5, field.vec_bytes(1 << 18))
    seen = set()
    for k in range(3):
        b = memory.chunked_block(shape, device=dev(), pooled=False)
        assert b.data_ptr() not in seen
        seen.add(b.data_ptr())
        junk = [torch.full((shape[0] * shape[1],), 7 + j, dtype=torch.uint8, device=dev()) for j in range(3)]
        b.fill_(0xA0 + k)  # after torch's new segments: no torch allocation shares the block's pages
        torch.cuda.synchronize()
        assert int((b != 0xA0 + k).sum().item()) == 0
        assert all(int((x != 7 + j).sum().item()) == 0 for j, x in enumerate(junk))
        del b, junk
        gc.collect()
    st = memory.pool_stats()
    assert st["idle_blocks"] == 0


def test_share_block_write_rate_probe():
    """A new share block of PROBE_MIN_BYTES or more is write-rate probed and
    the kept block records its rate; the rejected tries are freed; an idle
    block is reused without a new probe."""
    memory.empty_cache()
    s0 = memory.pool_stats()
    nb = memory.PROBE_MIN_BYTES + (4 << 20)
    b = memory.share_block((nb,), dev())
    st = memory.pool_stats()
    assert st["probed"] >= s0["probed"] + 1
    assert st["allocs"] - s0["allocs"] == st["probed"] - s0["probed"]
    assert st["rejected"] - s0["rejected"] == st["probed"] - s0["probed"] - 1
    assert memory.block_rate(b) is not None and memory.block_rate(b) > 1e11
    b.fill_(3)
    assert int(b[-1].item()) == 3 and int(b[0].item()) == 3
    ptr = b.data_ptr()
    del b
    gc.collect()
    c = memory.share_block((nb,), dev())  # the idle block comes back, no new probe
    assert c.data_ptr() == ptr and memory.pool_stats()["probed"] == st["probed"]
    assert memory.block_rate(c) is not None
    small = memory.share_block((memory.CHUNKED_MIN_BYTES - 4096,), dev())  # below CHUNKED_MIN_BYTES: torch.empty
    assert memory.block_rate(small) is None
    del c, small
    gc.collect()
    memory.empty_cache()


def test_block_free_rejects_foreign_pointer():
    x = torch.empty(16, dtype=torch.uint8, device=dev())
    assert _native.lib().dn_block_free(x.data_ptr()) == _native.DN_ERR_ARG


# ------------------------------------------------------------ stream-ordered reuse
_cycles_per_ms = []


def _busy(ms: float) -> None:
    """Keep the current stream busy for about `ms` (torch.cuda._sleep,
    calibrated once: its cycle count is a clock whose rate we do not assume)."""
    if not _cycles_per_ms:
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        torch.cuda._sleep(10_000_000)
        e.record()
        e.synchronize()
        _cycles_per_ms.append(10_000_000 / max(s.elapsed_time(e), 1e-3))
    torch.cuda._sleep(int(ms * _cycles_per_ms[0]))


def _ref_shares(seed, sec, t, n):
    """make_shares_vec into torch.empty memory on the default stream."""
    ref = shamir.SecretShare(t)
    ref.random.seed(seed)
    out = torch.empty((n, field.vec_bytes(sec.numel())), dtype=torch.uint8, device=dev())
    ref.make_shares_vec(sec, n, out=out)
    torch.cuda.synchronize()
    return out


def test_share_block_not_reused_while_another_stream_still_reads_it(monkeypatch):
    """The returned shares belong to the caller (shamir.py:62-66): a block
    freed while stream A still has work queued on it is not handed to a
    request on stream B — A's queued read sees A's shares, B gets its own.
    (Blocks unprobed here: a probe that rejects a block frees it, and the
    free may wait for the device, i.e. for A's queued work — the race this
    test needs would be lost on a box where the first try is rejected.)"""
    monkeypatch.setattr(memory, "PROBE_MIN_BYTES", 1 << 62)
    memory.empty_cache()
    N = 1 << 18
    sec_a = torch.randint(-(1 << 62), 1 << 62, (N,), dtype=torch.int64, device=dev())
    sec_b = torch.randint(-(1 << 62), 1 << 62, (N,), dtype=torch.int64, device=dev())
    want_a, want_b = _ref_shares(21, sec_a, 3, 5), _ref_shares(22, sec_b, 3, 5)
    sa, sb = torch.cuda.Stream(), torch.cuda.Stream()
    a, b = shamir.SecretShare(3), shamir.SecretShare(3)
    a.random.seed(21)
    b.random.seed(22)
    s0 = memory.pool_stats()
    with torch.cuda.stream(sa):
        out_a = a.make_shares_vec(sec_a, 5)  # a pooled block, used on stream A
        ptr_a = out_a.data_ptr()
        _busy(3000)
        kept = out_a.clone()  # queued on A behind the sleep: reads the block later
        del out_a
        gc.collect()  # the block goes idle with A's read still queued
    assert memory.pool_stats()["idle_blocks"] == s0["idle_blocks"] + 1
    with torch.cuda.stream(sb):
        out_b = b.make_shares_vec(sec_b, 5)  # same size, another stream
    a_busy = not sa.query()
    torch.cuda.synchronize()
    assert a_busy, "stream A finished before the request on B: the test did not race"
    assert out_b.data_ptr() != ptr_a
    assert memory.pool_stats()["busy_skips"] > s0["busy_skips"]
    assert torch.equal(kept, want_a) and torch.equal(out_b, want_b)
    del out_b, kept
    gc.collect()
    memory.empty_cache()


def test_share_block_reused_at_once_on_the_same_stream():
    memory.empty_cache()
    shape = (5, field.vec_bytes(1 << 18))
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        x = memory.chunked_block(shape, device=dev())
        ptr = x.data_ptr()
        _busy(500)
        x.fill_(1)
        del x
        gc.collect()
        y = memory.chunked_block(shape, device=dev())  # stream order covers the queued fill
        assert y.data_ptr() == ptr
        y.fill_(2)
    torch.cuda.synchronize()
    assert int((y != 2).sum().item()) == 0
    del y
    gc.collect()
    memory.empty_cache()


def test_busy_idle_block_taken_with_a_device_wait():
    """The out-of-memory fallback: a request on B takes a block A still uses,
    and B waits for A's recorded event on the device (dn_block_acquire wait=1):
    B's write lands after A's queued read."""
    memory.empty_cache()
    shape = (5, field.vec_bytes(1 << 18))
    sa, sb = torch.cuda.Stream(), torch.cuda.Stream()
    with torch.cuda.stream(sa):
        x = memory.chunked_block(shape, device=dev())
        x.fill_(0x5A)
        key = (dev().index, x.numel(), memory.CHUNK_BYTES)
        _busy(3000)
        kept = x.clone()
        del x
        gc.collect()
    raw_b = sb.cuda_stream
    assert memory._take_idle(key, raw_b) is None  # not ready for B
    ptr = memory._take_idle(key, raw_b, wait=True)
    assert ptr is not None
    with torch.cuda.stream(sb):
        blk = memory._Block(ptr, key, shape, True, raw_b)
        y = torch.as_tensor(blk, device=dev())
        y.fill_(0xC3)  # ordered after A's clone by the event wait
    torch.cuda.synchronize()
    assert int((kept != 0x5A).sum().item()) == 0 and int((y != 0xC3).sum().item()) == 0
    del y, blk, kept
    gc.collect()
    memory.empty_cache()


def test_record_stream_orders_reuse_after_a_second_stream():
    memory.empty_cache()
    shape = (5, field.vec_bytes(1 << 18))
    sa, sc = torch.cuda.Stream(), torch.cuda.Stream()
    with torch.cuda.stream(sa):
        x = memory.chunked_block(shape, device=dev())
        x.fill_(0x11)
        key = (dev().index, x.numel(), memory.CHUNK_BYTES)
    torch.cuda.synchronize()
    with torch.cuda.stream(sc):  # the caller hands the block to stream C
        _busy(3000)
        kept = x.clone()
    memory.record_stream(x, sc)
    del x
    gc.collect()
    assert memory._take_idle(key, sa.cuda_stream) is None  # C's queued read is pending
    torch.cuda.synchronize()
    p = memory._take_idle(key, sa.cuda_stream)
    assert p is not None  # completed: free to take
    memory._free_ptr(p)
    assert int((kept != 0x11).sum().item()) == 0
    memory.empty_cache()


def test_retry_acquire_keeps_every_streams_order():
    """a block used on streams A and B goes idle with both
    reads queued.  A request on A must not take it while B is busy — and the
    refused request must leave A's record intact, so that once B is done a
    request on a third stream C still waits for A (dn_block_acquire checks
    every stream before it clears any).  Then C's write lands after A's read."""
    memory.empty_cache()
    shape = (5, field.vec_bytes(1 << 18))
    sa, sb, sc = torch.cuda.Stream(), torch.cuda.Stream(), torch.cuda.Stream()
    with torch.cuda.stream(sa):
        x = memory.chunked_block(shape, device=dev())
        x.fill_(0x3C)
        key = (dev().index, x.numel(), memory.CHUNK_BYTES)
    torch.cuda.synchronize()
    with torch.cuda.stream(sa):
        _busy(3000)
        kept_a = x.clone()  # A's read, queued behind 3 s
    with torch.cuda.stream(sb):
        _busy(300)
        kept_b = x.clone()  # B's read, queued behind 0.3 s
    memory.record_stream(x, sb)
    del x
    gc.collect()
    assert memory._take_idle(key, sa.cuda_stream) is None  # B still busy: RETRY, nothing changed
    sb.synchronize()
    a_busy = not sa.query()
    assert memory._take_idle(key, sc.cuda_stream) is None  # A's read is still pending
    assert a_busy, "stream A finished before the request on C: the test did not race"
    ptr = memory._take_idle(key, sc.cuda_stream, wait=True)  # C waits for A on the device
    assert ptr is not None
    with torch.cuda.stream(sc):
        blk = memory._Block(ptr, key, shape, True, sc.cuda_stream)
        y = torch.as_tensor(blk, device=dev())
        y.fill_(0xC3)
    torch.cuda.synchronize()
    assert int((kept_a != 0x3C).sum().item()) == 0 and int((kept_b != 0x3C).sum().item()) == 0
    assert int((y != 0xC3).sum().item()) == 0
    del y, blk, kept_a, kept_b
    gc.collect()
    memory.empty_cache()


def test_unpooled_allocate_free_loop_counts_retired_space(monkeypatch):
    """every freed block retires its range; the count is
    exact, and past RETIRE_BUDGET share_block hands out torch.empty memory
    instead of mapping (and later retiring) new ranges."""
    memory.empty_cache()
    shape = (2, 32 << 20)  # 64 MiB: a chunked share block
    r0 = memory.retired_bytes()
    for _ in range(20):
        x = memory.chunked_block(shape, device=dev(), pooled=False)
        x.fill_(7)
        del x
        gc.collect()
    torch.cuda.synchronize()
    assert memory.retired_bytes() - r0 == 20 * (64 << 20)
    monkeypatch.setattr(memory, "RETIRE_BUDGET", memory.retired_bytes() + (32 << 20))
    before = memory.pool_stats()["va_fallbacks"]
    y = memory.share_block(shape, dev())
    assert memory.pool_stats()["va_fallbacks"] == before + 1 and memory.block_rate(y) is None
    y.fill_(1)
    assert int(y.sum().item()) == y.numel()
    del y
    memory.empty_cache()


def test_make_shares_vec_t4_loop_on_a_side_stream_equals_host_draw():
    """t = 4 takes the draw-then-split path: its coefficient block (pooled,
    >= 64 MiB here) is dropped right after the split is queued, and every
    iteration's output block goes back to the pool.  On a side stream, each
    call equals the host draw + split of the same generator."""
    memory.empty_cache()
    N, t, n = 1 << 19, 4, 6
    assert (t - 1) * field.vec_bytes(N) >= memory.CHUNKED_MIN_BYTES
    sec = torch.randint(-(1 << 62), 1 << 62, (N,), dtype=torch.int64, device=dev())
    a, ref = shamir.SecretShare(t), shamir.SecretShare(t)
    a.random.seed(5)
    ref.random.seed(5)
    s = torch.cuda.Stream()
    outs = []
    s0 = memory.pool_stats()
    with torch.cuda.stream(s):
        for _ in range(4):
            out = a.make_shares_vec(sec, n)
            outs.append(out.clone())
            del out
            gc.collect()
    torch.cuda.synchronize()
    assert memory.pool_stats()["reuses"] > s0["reuses"]
    for got in outs:
        co = torch.from_numpy(_native.mt_draw_coeffs(ref.random, N, t - 1)).to(dev())
        want = torch.empty_like(got)
        _native.split_u64(sec, co, want, N, t, n)
        assert torch.equal(got, want)
    assert a.random.getstate() == ref.random.getstate()
    memory.empty_cache()


@pytest.mark.skipif(torch.cuda.device_count() < 2, reason="needs two HIP devices")
def test_block_free_waits_on_the_blocks_own_device():
    """dn_block_free of a block on cuda:1 while cuda:0 is current: the wait is
    on cuda:1's work (its recorded event), the free succeeds and cuda:0 stays
    current."""
    memory.empty_cache()
    torch.cuda.set_device(0)
    d1 = torch.device("cuda", 1)
    x = memory.chunked_block((memory.CHUNKED_MIN_BYTES,), device=d1, pooled=False)
    with torch.cuda.device(1):
        _busy(500)
        x.fill_(3)
    del x
    gc.collect()
    assert torch.cuda.current_device() == 0
    torch.cuda.synchronize(1)
