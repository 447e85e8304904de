"""memory.share_block's placement policy (delta_node/crypto/shamir/memory.py),
host logic only: which of the probed blocks is kept and which are freed.
The device calls (dn_block_alloc, the timed probe write, dn_block_free) are
replaced by fakes with scripted rates, so this runs without a GPU."""
import types

import pytest

from delta_node.crypto.shamir import memory


class Fake:
    def __init__(self, rates):
        self.rates = list(rates)
        self.next_ptr = 0x1000
        self.rate_of = {}
        self.freed = []

    def alloc(self, nbytes, chunk, index):
        if not self.rates:
            raise RuntimeError("out of memory")
        p = self.next_ptr
        self.next_ptr += 0x1000
        self.rate_of[p] = self.rates.pop(0)
        return p

    def rate(self, ptr, nbytes, dev, shape):
        return self.rate_of[ptr]

    def free(self, ptr, streams=()):
        self.freed.append(ptr)


@pytest.fixture
def fake(monkeypatch):
    def make(rates):
        f = Fake(rates)
        monkeypatch.setattr(memory, "_alloc_raw", f.alloc)
        monkeypatch.setattr(memory, "_write_rate", f.rate)
        monkeypatch.setattr(memory, "_free_ptr", f.free)
        monkeypatch.setattr(memory, "_best_rate", {})
        monkeypatch.setattr(memory, "_rates", {})
        monkeypatch.setattr(memory, "_current_stream", lambda index: 0)
        monkeypatch.setattr(memory, "_mem_info", lambda index: (1 << 50, 1 << 50))
        monkeypatch.setattr(memory, "PROBE_FIRST_SMALL", 2)  # the tests below script two first tries
        monkeypatch.setattr(memory, "_retired", lambda: 0)
        return f
    return make


DEV = types.SimpleNamespace(index=0)
SHAPE = (5, 16896 * 1024)
NB = SHAPE[0] * SHAPE[1]


def test_first_block_is_the_faster_of_two(fake):
    f = fake([5.0, 7.0, 9.0])
    p = memory._alloc_probed(NB, 2 << 20, DEV, SHAPE)
    assert f.rate_of[p] == 7.0 and f.freed == [0x1000] and f.rates == [9.0]
    assert memory._best_rate[(0, 5, NB.bit_length())] == 7.0 and memory._rates[p] == 7.0


def test_fast_class_block_kept_at_once(fake):
    """The first block of a class whose tiled (split-order) probe reaches
    PROBE_FAST is kept without a second try; later blocks compare with the
    best rate seen."""
    fast = memory.PROBE_FAST
    f = fake([fast * 1.01, fast * 1.2, fast * 1.02, fast * 1.25])
    p = memory._alloc_probed(NB, 2 << 20, DEV, SHAPE)
    assert f.rate_of[p] == fast * 1.01 and f.freed == [] and f.rates == [fast * 1.2, fast * 1.02, fast * 1.25]
    memory._best_rate[(0, 5, NB.bit_length())] = fast * 1.3  # a faster block was seen since
    q = memory._alloc_probed(NB, 2 << 20, DEV, SHAPE)  # 1.2 and 1.02 fall short of 0.96 x 1.3; 1.25 passes
    assert f.rate_of[q] == fast * 1.25 and f.rates == []
    g = fake([fast * 1.01, fast * 1.2])  # a linear-fill probe (untiled shape): the faster of two
    q = memory._alloc_probed(NB, 2 << 20, DEV, (NB,))
    assert g.rate_of[q] == fast * 1.2 and len(g.freed) == 1


def test_later_block_kept_when_close_to_the_best(fake):
    f = fake([7.0, 6.0, 6.8])
    memory._alloc_probed(NB, 2 << 20, DEV, SHAPE)  # best 7.0 (the first of two tries)
    p = memory._alloc_probed(NB, 2 << 20, DEV, SHAPE)  # 6.8 >= 0.96 * 7.0: kept at once
    assert f.rate_of[p] == 6.8 and f.rates == []


BIG = (5, 16896 * 16384)  # 1.38 GB: a 2^22-element share block
NBIG = BIG[0] * BIG[1]


def test_slow_block_redrawn_up_to_the_try_limit(fake):
    slow = [5.0, 5.5, 6.5] + [5.2] * (memory.PROBE_TRIES - 3)
    f = fake([7.0, 6.0] + slow + [9.9])
    memory._alloc_probed(NBIG, 2 << 20, DEV, BIG)  # keeps 7.0, frees 6.0
    p = memory._alloc_probed(NBIG, 2 << 20, DEV, BIG)  # PROBE_TRIES tries, none close: keeps 6.5
    assert f.rate_of[p] == 6.5
    assert sorted(f.rate_of[q] for q in f.freed) == sorted([6.0] + [r for r in slow if r != 6.5])
    assert f.rates == [9.9]  # PROBE_TRIES blocks at most


def test_tries_bounded_by_free_memory(fake, monkeypatch):
    f = fake([7.0, 6.0, 5.0, 5.5, 6.5, 9.9])
    memory._alloc_probed(NBIG, 2 << 20, DEV, BIG)  # keeps 7.0, frees 6.0
    monkeypatch.setattr(memory, "_mem_info", lambda index: (memory.POOL_MIN_FREE + 2 * NBIG + 1, 288 << 30))
    p = memory._alloc_probed(NBIG, 2 << 20, DEV, BIG)  # room for two tries beyond the margin
    assert f.rate_of[p] == 5.5 and f.rates == [6.5, 9.9]


def test_small_blocks_get_more_tries(fake):
    rates = [7.0, 6.0] + [5.0] * (memory.PROBE_TRIES_SMALL - 1) + [6.9, 9.9]
    f = fake(rates)
    memory._alloc_probed(NB, 2 << 20, DEV, SHAPE)  # keeps 7.0
    p = memory._alloc_probed(NB, 2 << 20, DEV, SHAPE)  # 11 slow tries, then 6.9 >= 0.96 * 7.0
    assert f.rate_of[p] == 6.9 and f.rates == [9.9]


def test_rates_compare_within_a_row_count(fake):
    f = fake([9.0, 9.5, 5.0, 5.1])
    memory._alloc_probed(NB, 2 << 20, DEV, (2, SHAPE[1]))  # coefficient-block class: best 9.5
    p = memory._alloc_probed(NB, 2 << 20, DEV, SHAPE)  # share-block class starts fresh: best of two
    assert f.rate_of[p] == 5.1 and memory._best_rate[(0, 5, NB.bit_length())] == 5.1


def test_rates_compare_within_a_size_class(fake):
    f = fake([9.0, 9.5, 5.0, 5.1])
    memory._alloc_probed(NB // 8, 2 << 20, DEV, (5, SHAPE[1] // 8))  # a small 5-row block: best 9.5
    p = memory._alloc_probed(NB, 2 << 20, DEV, SHAPE)  # a large one is its own class: best of two
    assert f.rate_of[p] == 5.1 and f.rates == []


def test_budget_limits_tries_for_huge_blocks(fake):
    f = fake([1.0, 2.0, 3.0])
    huge = memory.PROBE_BUDGET  # one try fits the budget
    p = memory._alloc_probed(huge, 2 << 20, DEV, (1, huge))
    assert f.rate_of[p] == 1.0 and f.freed == []


def test_out_of_memory_keeps_the_best_so_far(fake):
    f = fake([7.0])  # the second try of the first block fails to allocate
    p = memory._alloc_probed(NB, 2 << 20, DEV, SHAPE)
    assert f.rate_of[p] == 7.0 and f.freed == []
    g = fake([])
    with pytest.raises(RuntimeError):
        memory._alloc_probed(NB, 2 << 20, DEV, SHAPE)
    assert g.freed == []


# ---------------------------------------------------------------- the idle pool
class FakeLib:
    """dn_block_* with scripted stream events: `busy` holds the pointers whose
    recorded uses on another stream have not completed."""

    def __init__(self):
        self.busy = set()
        self.recorded = []
        self.acquired = []
        self.freed = []

    def dn_block_record(self, ptr, stream):
        if ptr in self.fail_record:
            return memory._native.DN_ERR_HIP
        self.recorded.append((ptr, stream or 0))
        return 0

    def dn_last_error(self):
        return b"scripted HIP error"

    def dn_block_acquire(self, ptr, stream, wait):
        if ptr in self.busy and not wait:
            return memory._native.DN_ERR_RETRY
        self.acquired.append((ptr, stream or 0, wait))
        return 0

    def dn_block_free(self, ptr):
        self.freed.append(ptr)
        return 0

    fail_record = ()


@pytest.fixture
def pool(monkeypatch):
    L = FakeLib()
    state = {"free": 100 << 30}
    monkeypatch.setattr(memory._native, "lib", lambda: L)
    monkeypatch.setattr(memory, "_idle", {})
    monkeypatch.setattr(memory, "_idle_bytes", 0)
    monkeypatch.setattr(memory, "_rates", {})
    monkeypatch.setattr(memory, "_live", {})
    monkeypatch.setattr(memory, "_mem_info", lambda index: (state["free"], 288 << 30))
    L.synced = []
    monkeypatch.setattr(memory, "_sync_device", lambda index: L.synced.append(index))
    L.state = state
    return L


def idle(key, ptr):
    """Put a block in the idle list as _Block.__del__ does."""
    b = memory._Block(ptr, key, (key[1],), True, 7)
    del b


KEY = (0, 1 << 30, 2 << 20)


def test_block_going_idle_records_every_stream_it_used(pool):
    b = memory._Block(0x100, KEY, (KEY[1],), True, 7)
    b.streams.add(9)
    del b
    assert sorted(pool.recorded) == [(0x100, 7), (0x100, 9)]
    assert memory._idle[KEY] and memory._idle_bytes == KEY[1]


def test_idle_block_reused_only_when_ready_for_the_stream(pool):
    idle(KEY, 0x100)
    pool.busy.add(0x100)  # another stream's work on it is still queued
    assert memory._take_idle(KEY, 5) is None
    assert memory._stats["busy_skips"] >= 1 and memory._idle_bytes == KEY[1]
    pool.busy.clear()  # its event completed (or the request is on the same stream)
    assert memory._take_idle(KEY, 5) == 0x100
    assert pool.acquired[-1] == (0x100, 5, 0) and memory._idle_bytes == 0


def test_busy_idle_block_taken_with_a_device_wait_only_on_request(pool):
    idle(KEY, 0x100)
    pool.busy.add(0x100)
    assert memory._take_idle(KEY, 5, wait=True) == 0x100
    assert pool.acquired[-1] == (0x100, 5, 1)


def test_newest_ready_idle_block_first(pool):
    idle(KEY, 0x100)
    idle(KEY, 0x200)
    pool.busy.add(0x200)
    assert memory._take_idle(KEY, 5) == 0x100


def test_block_not_pooled_when_the_device_is_short_of_memory(pool):
    pool.state["free"] = memory.POOL_MIN_FREE - 1
    idle(KEY, 0x100)
    assert pool.freed == [0x100] and KEY not in memory._idle


def test_idle_cap(pool, monkeypatch):
    monkeypatch.setattr(memory, "POOL_IDLE_BYTES", 3 << 30)
    for k in range(5):
        idle(KEY, 0x100 * (k + 1))
    assert len(memory._idle[KEY]) == 3 and pool.freed == [0x400, 0x500]


def test_trim_releases_oldest_idle_blocks_until_the_new_block_fits(pool):
    k2 = (0, 2 << 30, 2 << 20)
    idle(KEY, 0x100)  # oldest
    idle(k2, 0x200)
    idle(KEY, 0x300)
    pool.state["free"] = memory.POOL_MIN_FREE + (1 << 30)
    memory._trim_for(3 << 30, 0)  # needs 2 GiB more: the two oldest go
    assert pool.freed == [0x100, 0x200] and memory._idle == {KEY: [memory._idle[KEY][0]]}
    assert memory._idle[KEY][0][1] == 0x300 and memory._idle_bytes == KEY[1]


def test_empty_cache_releases_every_idle_block(pool):
    idle(KEY, 0x100)
    idle((0, 2 << 30, 2 << 20), 0x200)
    memory.empty_cache()
    assert sorted(pool.freed) == [0x100, 0x200] and memory._idle == {} and memory._idle_bytes == 0


def test_record_stream_adds_a_stream_to_the_live_block(pool):
    b = memory._Block(0x1000, KEY, (KEY[1],), True, 7)
    memory._live[0x1000] = __import__("weakref").ref(b)
    view = types.SimpleNamespace(data_ptr=lambda: 0x1000 + 4096)
    memory.record_stream(view, types.SimpleNamespace(cuda_stream=11))
    assert b.streams == {7, 11}
    outside = types.SimpleNamespace(data_ptr=lambda: 0x1000 + KEY[1])
    memory.record_stream(outside, 12)
    assert b.streams == {7, 11}


def test_first_small_block_is_the_fastest_of_probe_first_small(fake, monkeypatch):
    f = fake([5.0, 7.0, 6.0, 7.5, 9.0])
    monkeypatch.setattr(memory, "PROBE_FIRST_SMALL", 4)
    p = memory._alloc_probed(NB, 2 << 20, DEV, SHAPE)  # under 1 GiB: the fastest of four
    assert f.rate_of[p] == 7.5 and len(f.freed) == 3 and f.rates == [9.0]
    g = fake([5.0, 7.0, 9.0])
    q = memory._alloc_probed(NBIG, 2 << 20, DEV, BIG)  # 1 GiB and up: the faster of PROBE_FIRST = 2
    assert g.rate_of[q] == 7.0 and g.rates == [9.0]


def test_failed_record_frees_the_block_after_a_device_wait(pool):
    """ADVICE/VERDICT r05: a block whose event cannot be recorded is neither
    pooled nor leaked — its device drains, then it is freed, and counted."""
    before = memory._stats["record_failures"]
    pool.fail_record = {0x100}
    b = memory._Block(0x100, KEY, (KEY[1],), True, 7)
    del b
    assert pool.freed == [0x100] and pool.synced == [0]
    assert KEY not in memory._idle and memory._idle_bytes == 0
    assert memory._stats["record_failures"] == before + 1


def test_time_budget_stops_the_tries(fake, monkeypatch):
    """Every try slow: the request stops once its tries plus the frees they
    imply (at the measured free cost of that size) would pass
    PROBE_TIME_BUDGET, and keeps the best block so far (the cold worst case
    stays bounded)."""
    f = fake([7.0, 6.0] + [5.0, 5.1, 5.2, 5.3, 5.4, 5.5, 5.6, 5.7] + [9.9])
    memory._alloc_probed(NBIG, 2 << 20, DEV, BIG)  # best 7.0
    monkeypatch.setattr(memory, "_free_secs", {NBIG: 0.010})  # a free of this size took 10 ms
    clock = iter([0.0] + [0.005 * k for k in range(1, 100)])  # each try takes 5 ms
    monkeypatch.setattr(memory.time, "perf_counter", lambda: next(clock))
    before = memory._stats["budget_stops"]
    p = memory._alloc_probed(NBIG, 2 << 20, DEV, BIG)
    # after try k (k = 1..): 5k ms spent + 5 ms next + 10k ms of frees; k = 4 passes 50 ms
    assert f.rate_of[p] == 5.3 and f.rates[0] == 5.4 and memory._stats["budget_stops"] == before + 1
    g = fake([7.0, 6.0] + [5.0, 5.1, 5.2] + [9.9])  # no free measured yet: a free costs a try
    memory._alloc_probed(NBIG, 2 << 20, DEV, BIG)
    monkeypatch.setattr(memory, "_free_secs", {})
    clock2 = iter([0.0] + [0.02 * k for k in range(1, 100)])  # 20 ms tries
    monkeypatch.setattr(memory.time, "perf_counter", lambda: next(clock2))
    q = memory._alloc_probed(NBIG, 2 << 20, DEV, BIG)  # 20 + 20 + 20 > 50 after the first
    assert g.rate_of[q] == 5.0 and g.rates[0] == 5.1


def test_retire_budget_limits_the_tries(fake, monkeypatch):
    """Rejected tries retire their ranges: a request never plans more tries
    than the address-space budget has room for."""
    f = fake([7.0, 6.0, 5.0, 5.1, 5.2, 9.9])
    memory._alloc_probed(NBIG, 2 << 20, DEV, BIG)  # best 7.0
    monkeypatch.setattr(memory, "_retired", lambda: memory.RETIRE_BUDGET - 2 * NBIG)
    p = memory._alloc_probed(NBIG, 2 << 20, DEV, BIG)
    assert f.rate_of[p] == 5.1 and f.rates == [5.2, 9.9]  # two tries


def test_share_block_past_the_retire_budget_is_torch_memory(monkeypatch):
    import torch

    calls = []
    monkeypatch.setattr(memory, "_device_index", lambda device: torch.device("cpu"))
    monkeypatch.setattr(memory, "chunked_block", lambda *a, **k: calls.append(a) or "chunked")
    monkeypatch.setattr(memory, "_idle", {})
    monkeypatch.setattr(memory, "_retired", lambda: 0)
    assert memory.share_block((2, 64 << 20)) == "chunked"
    monkeypatch.setattr(memory, "_retired", lambda: memory.RETIRE_BUDGET - (64 << 20))
    before = memory._stats["va_fallbacks"]
    t = memory.share_block((2, 64 << 20))
    assert isinstance(t, torch.Tensor) and t.shape == (2, 64 << 20) and len(calls) == 1
    assert memory._stats["va_fallbacks"] == before + 1
