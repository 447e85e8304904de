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

    def free(self, ptr):
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
        return f
    return make


DEV = types.SimpleNamespace(index=0)
SHAPE = (5, 16896 * 1024)
NB = SHAPE[0] * SHAPE[1]


def test_first_block_is_the_faster_of_two(fake):
    f = fake([5.0, 7.0, 9.0])
    p = memory._alloc_probed(NB, 2 << 20, DEV, SHAPE)
    assert f.rate_of[p] == 7.0 and f.freed == [0x1000] and f.rates == [9.0]
    assert memory._best_rate[(0, 5)] == 7.0 and memory._rates[p] == 7.0


def test_later_block_kept_when_close_to_the_best(fake):
    f = fake([7.0, 6.0, 6.8])
    memory._alloc_probed(NB, 2 << 20, DEV, SHAPE)  # best 7.0 (the first of two tries)
    p = memory._alloc_probed(NB, 2 << 20, DEV, SHAPE)  # 6.8 >= 0.96 * 7.0: kept at once
    assert f.rate_of[p] == 6.8 and f.rates == []


def test_slow_block_redrawn_up_to_the_try_limit(fake):
    f = fake([7.0, 6.0, 5.0, 5.5, 6.5, 5.2, 9.9])
    memory._alloc_probed(NB, 2 << 20, DEV, SHAPE)  # keeps 7.0, frees 6.0
    p = memory._alloc_probed(NB, 2 << 20, DEV, SHAPE)  # 5.0, 5.5, 6.5, 5.2: none close, keeps 6.5
    assert f.rate_of[p] == 6.5
    assert sorted(f.rate_of[q] for q in f.freed) == [5.0, 5.2, 5.5, 6.0]
    assert f.rates == [9.9]  # PROBE_TRIES blocks at most


def test_rates_compare_within_a_row_count(fake):
    f = fake([9.0, 9.5, 5.0, 5.1])
    memory._alloc_probed(NB, 2 << 20, DEV, (2, SHAPE[1]))  # coefficient-block class: best 9.5
    p = memory._alloc_probed(NB, 2 << 20, DEV, SHAPE)  # share-block class starts fresh: best of two
    assert f.rate_of[p] == 5.1 and memory._best_rate[(0, 5)] == 5.1


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
