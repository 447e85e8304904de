"""Share-block memory (delta_node.crypto.shamir.memory, csrc/vmm_block.cpp):
blocks of 2 MiB physical chunks, pooled, aliased by torch tensors through
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
    assert st["allocs"] + st["reuses"] == s0["allocs"] + s0["reuses"] + 1
    want = torch.empty_like(out)
    b.make_shares_vec(sec, 5, out=want)
    assert torch.equal(out, want) and a.random.getstate() == b.random.getstate()
    small = a.make_shares_vec(sec[:1000], 5)  # below the threshold: torch.empty
    assert memory.pool_stats()["allocs"] + memory.pool_stats()["reuses"] == st["allocs"] + st["reuses"]
    assert tuple(small.shape) == (5, field.vec_bytes(1000))


def test_freed_block_address_is_never_reused():
    """A freed block's virtual range is retired (csrc/vmm_block.cpp): the next
    block lands elsewhere, and its bytes stay put under later allocations.
    (Before: a new block at a freed block's address had its contents change
    under unrelated torch allocations — scripts/msv_block_debug.py, r04i.)"""
    memory.empty_cache()
    shape = (5, field.vec_bytes(1 << 18))
    seen = set()
    for k in range(3):
        b = memory.chunked_block(shape, device=dev(), pooled=False)
        assert b.data_ptr() not in seen
        seen.add(b.data_ptr())
        b.fill_(0xA0 + k)
        junk = [torch.full((shape[0] * shape[1],), 7, dtype=torch.uint8, device=dev()) for _ in range(3)]
        torch.cuda.synchronize()
        assert int((b != 0xA0 + k).sum().item()) == 0
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
    small = memory.share_block((memory.CHUNKED_MIN_BYTES + 4096,), dev())  # below PROBE_MIN_BYTES: not probed
    assert memory.block_rate(small) is None
    del c, small
    gc.collect()
    memory.empty_cache()


def test_block_free_rejects_foreign_pointer():
    x = torch.empty(16, dtype=torch.uint8, device=dev())
    assert _native.lib().dn_block_free(x.data_ptr()) == _native.DN_ERR_ARG
