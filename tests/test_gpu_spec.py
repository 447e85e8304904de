"""The device draw's speculation on loops of equal draws (DN_MT_SPEC,
csrc/mt19937_device.hip): a call that continues the previous one (same size,
starting where it ended) also computes the jump windows of a next draw of that
size starting where it ends, and a matching next call uses them instead of
jumping.  Invisible but
for time: every call here equals the sequential host draw (the reference's
randint sequence, shamir.py:59-61) + split byte for byte, with the same final
random.Random state — on hits, on misses (state touched in between, another
size in between, a forced rejected draw) and across streams — and the
counters show which path ran."""
import random

import numpy as np
import pytest
import torch

from delta_node.crypto import shamir
from delta_node.crypto.shamir import _native, field
from golden.fixtures import secrets_int64

pytestmark = pytest.mark.gpu


def dev():
    return torch.device("cuda", torch.cuda.current_device())


@pytest.fixture(scope="module", autouse=True)
def _native_loaded():
    assert torch.cuda.is_available(), "GPU tests need a HIP device"
    _native.lib()


def host_shares(rng: random.Random, sec: torch.Tensor, n: int, t: int, n_shares: int) -> torch.Tensor:
    """The sequential host draw (C restatement of the reference's draws) + the split."""
    co = torch.from_numpy(_native.mt_draw_coeffs(rng, n, t - 1)).to(sec.device)
    want = torch.zeros((n_shares, field.vec_bytes(n)), dtype=torch.uint8, device=sec.device)
    _native.split_u64(sec, co, want, n, t, n_shares)
    return want


def device_shares(ss: shamir.SecretShare, sec: torch.Tensor, n: int, n_shares: int) -> torch.Tensor:
    out = torch.zeros((n_shares, field.vec_bytes(n)), dtype=torch.uint8, device=sec.device)  # padding stays 0
    assert _native.mt_split_device(ss.random, sec, out, n, ss.threshold, n_shares)
    return out


def valid_limbs(block: torch.Tensor, n: int) -> np.ndarray:
    h = block.cpu().numpy()
    return np.stack([field.vec_to_limbs(h[r], n) for r in range(h.shape[0])])


# the product library speculates after the generation on draws of at least
# 2^23 coefficients (DN_MT_SPEC_MIN) and beside it from 2^16 where the levels
# fit beside the generation (DN_MT_BESIDE_MIN); smaller draws are tested
# through the tuning build with the thresholds at 0 (every draw with jump
# levels speculates)
SPEC_MIN = 1 << 23


@pytest.fixture
def any_size(monkeypatch):
    monkeypatch.setenv("DN_MT_SPEC_MIN", "0")
    with _native.library(_native.TUNING_LIB):
        yield


def delta(before: dict, after: dict) -> dict:
    return {k: after[k] - before[k] for k in ("hits", "misses", "launched")}


@pytest.mark.parametrize("N,t,n,pre", [(40000, 3, 5, 0), ((1 << 20) + 77, 3, 5, 333), (1 << 23, 3, 5, 0),
                                       ((1 << 22) + 5, 5, 9, 600)])
def test_loop_of_equal_draws_hits_and_equals_host_draw(N, t, n, pre, monkeypatch):
    """Five equal calls: the third to fifth use speculated windows (the second
    launches the first speculation); each equals the host draw + split and
    leaves the same state — from a mid-array start, at sizes whose draws take
    the direct level, the radix levels and the 2^24-scale runtime level (the
    product library there, the tuning build below its threshold)."""
    if N * (t - 1) < SPEC_MIN:
        monkeypatch.setenv("DN_MT_SPEC_MIN", "0")
        with _native.library(_native.TUNING_LIB):
            _loop_case(N, t, n, pre)
    else:
        _loop_case(N, t, n, pre)


@pytest.mark.parametrize("N,t,n,pre,lib", [((1 << 20) + 77, 3, 5, 333, "product"), (1 << 19, 5, 9, 0, "product"),
                                           ((1 << 16) + 1, 3, 5, 5, "product"),
                                           (40000, 3, 5, 17, "tuning"), (5000, 5, 9, 600, "tuning"),
                                           ((1 << 21) + 9, 2, 3, 0, "tuning")])
def test_loop_beside_a_small_generation(N, t, n, pre, lib, monkeypatch):
    """Draws whose generation leaves a CU room for the jump levels' 83 KB
    workgroups (at most ~1000 3-of-5 substreams, of 2^12 draws or at most
    256 of 2^10) speculate beside the generation with those levels as they
    are, from the next call's W_idx jumped on a side stream: the product
    library from 2^16 coefficients (DN_MT_BESIDE_MIN; no speculation after the
    generation below 2^23), the
    tuning build with the threshold at 0 for the direct-level and radix-level
    shapes below it.  Every call equals the host draw + split."""
    if lib == "tuning":
        monkeypatch.setenv("DN_MT_BESIDE_MIN", "0")
        with _native.library(_native.TUNING_LIB):
            _loop_case(N, t, n, pre)
    else:
        _loop_case(N, t, n, pre)


def test_loop_of_coefficient_draws_beside(monkeypatch):
    """The coefficient draw (dn_mt19937_draw_coeffs_device, one-register
    rings) in a loop of equal draws of 2^20 + 5 elements x 2 coefficients:
    speculated beside the generation, every draw equal to the host's."""
    N, tm1 = (1 << 20) + 5, 2
    a, b = random.Random(77), random.Random(77)
    s0 = _native.mt_spec_stats()
    out = torch.zeros((tm1, field.vec_bytes(N)), dtype=torch.uint8, device=dev())  # padding stays 0
    for i in range(5):
        assert _native.mt_draw_coeffs_device(a, N, tm1, out)
        want = _native.mt_draw_coeffs(b, N, tm1)
        assert np.array_equal(out.cpu().numpy(), want), i
        assert a.getstate() == b.getstate(), i
    d = delta(s0, _native.mt_spec_stats())
    assert d["hits"] >= 3 and d["launched"] >= 4, d


def _loop_case(N, t, n, pre):
    sec = torch.from_numpy(secrets_int64(N % 977 + t, N)).to(dev())
    a, b = shamir.SecretShare(t), shamir.SecretShare(t)
    a.random.seed(N + pre)
    a.random.getrandbits(32 * pre)
    b.random.setstate(a.random.getstate())
    s0 = _native.mt_spec_stats()
    for i in range(5):
        got = device_shares(a, sec, N, n)
        want = host_shares(b.random, sec, N, t, n)
        assert torch.equal(got, want), (N, i)
        assert a.random.getstate() == b.random.getstate(), (N, i)
    d = delta(s0, _native.mt_spec_stats())
    assert d["hits"] >= 3 and d["launched"] >= 4, d


def test_state_touched_between_calls_misses(any_size):
    """random.Random used between two calls misses (the call compares the
    array and index it finds, and jumps itself); a state reseeded to the very
    one the speculation expected hits."""
    N, t, n = (1 << 20) + 3, 3, 5
    sec = torch.from_numpy(secrets_int64(5, N)).to(dev())
    a, b = shamir.SecretShare(t), shamir.SecretShare(t)
    a.random.seed(17)
    b.random.seed(17)
    for _ in range(2):  # the second call continues the first: it speculates
        assert torch.equal(device_shares(a, sec, N, n), host_shares(b.random, sec, N, t, n))
    s0 = _native.mt_spec_stats()
    assert s0["armed"]
    a.random.random()
    b.random.random()
    assert torch.equal(device_shares(a, sec, N, n), host_shares(b.random, sec, N, t, n))  # a miss
    s1 = _native.mt_spec_stats()
    assert delta(s0, s1)["misses"] == 1 and delta(s0, s1)["hits"] == 0 and not s1["armed"]
    assert torch.equal(device_shares(a, sec, N, n), host_shares(b.random, sec, N, t, n))  # continues: speculates
    assert _native.mt_spec_stats()["armed"]
    st = a.random.getstate()
    a.random.seed(99)
    a.random.setstate(st)  # the same state again: a hit
    assert torch.equal(device_shares(a, sec, N, n), host_shares(b.random, sec, N, t, n))
    s2 = _native.mt_spec_stats()
    assert delta(s1, s2)["hits"] == 1
    assert a.random.getstate() == b.random.getstate()


def test_other_sizes_and_kinds_in_between(any_size):
    """Sizes interleaved (each call misses the other's speculation), and the
    coefficient draw and the fused split of one draw size (t - 1 coefficients
    per element x elements) sharing a speculation: all equal the host draw."""
    a, b = shamir.SecretShare(3), shamir.SecretShare(3)
    a.random.seed(3)
    b.random.seed(3)
    N1, N2 = 300001, 70001
    sec = torch.from_numpy(secrets_int64(7, N1)).to(dev())
    for N in (N1, N1, N2, N1, N2, N2, N2):
        assert torch.equal(device_shares(a, sec[:N], N, 5), host_shares(b.random, sec[:N], N, 3, 5)), N
        assert a.random.getstate() == b.random.getstate()
    s0 = _native.mt_spec_stats()
    for _ in range(2):  # coefficient draws of N2 x 2, then a fused split of the same draw size
        got = torch.zeros((2, field.vec_bytes(N2)), dtype=torch.uint8, device=dev())
        assert _native.mt_draw_coeffs_device(a.random, N2, 2, got)
        want = torch.from_numpy(_native.mt_draw_coeffs(b.random, N2, 2)).to(dev())
        assert torch.equal(got, want)
    assert torch.equal(device_shares(a, sec[:N2], N2, 5), host_shares(b.random, sec[:N2], N2, 3, 5))
    assert a.random.getstate() == b.random.getstate()
    assert delta(s0, _native.mt_spec_stats())["hits"] >= 2


def test_forced_retry_disarms(monkeypatch, any_size):
    """A rejected draw (forced: tuning build's DN_MT_FORCE_RETRY) returns with
    the state untouched and arms nothing; make_shares_vec redoes it on the
    host, and the next device call, finding the host's final state, misses
    nothing it should not: same shares and state as the host draws."""
    N = 200003
    sec = torch.from_numpy(secrets_int64(8, N)).to(dev())
    if True:  # (the tuning build: any_size)
        a, b = shamir.SecretShare(3), shamir.SecretShare(3)
        a.random.seed(11)
        b.random.seed(11)
        for _ in range(2):
            assert torch.equal(device_shares(a, sec, N, 5), host_shares(b.random, sec, N, 3, 5))
        assert _native.mt_spec_stats()["armed"]
        monkeypatch.setenv("DN_MT_FORCE_RETRY", "1")
        got = a.make_shares_vec(sec, 5)  # device draw rejected -> host draw + split
        monkeypatch.delenv("DN_MT_FORCE_RETRY")
        assert not _native.mt_spec_stats()["armed"]
        want = host_shares(b.random, sec, N, 3, 5)
        assert np.array_equal(valid_limbs(got, N), valid_limbs(want, N))  # (the pooled block's padding is unspecified)
        assert a.random.getstate() == b.random.getstate()
        for _ in range(3):
            assert torch.equal(device_shares(a, sec, N, 5), host_shares(b.random, sec, N, 3, 5))
            assert a.random.getstate() == b.random.getstate()


def test_speculation_across_streams(any_size):
    """Calls alternating between torch's default stream and a side stream: the
    speculated windows are awaited on whichever stream the next call uses."""
    N = (1 << 20) + 1
    sec = torch.from_numpy(secrets_int64(9, N)).to(dev())
    a, b = shamir.SecretShare(3), shamir.SecretShare(3)
    a.random.seed(21)
    b.random.seed(21)
    st = torch.cuda.Stream()
    s0 = _native.mt_spec_stats()
    for i in range(6):
        if i % 2:
            with torch.cuda.stream(st):
                got = device_shares(a, sec, N, 5)
            st.synchronize()
        else:
            got = device_shares(a, sec, N, 5)
        assert torch.equal(got, host_shares(b.random, sec, N, 3, 5)), i
    assert a.random.getstate() == b.random.getstate()
    assert delta(s0, _native.mt_spec_stats())["hits"] >= 4


def test_speculation_off_and_below_threshold(monkeypatch):
    """DN_MT_SPEC=0 (tuning build) turns speculation off, and the product
    library does not speculate on draws below 2^23 coefficients: no launches,
    the same shares and states as the product library's speculating loop."""
    N = 1 << 22
    sec = torch.from_numpy(secrets_int64(10, N)).to(dev())
    a = shamir.SecretShare(3)
    a.random.seed(4)
    s0 = _native.mt_spec_stats()
    on = [device_shares(a, sec, N, 5) for _ in range(4)]
    assert delta(s0, _native.mt_spec_stats())["hits"] == 2
    monkeypatch.setenv("DN_MT_SPEC", "0")
    with _native.library(_native.TUNING_LIB):
        c = shamir.SecretShare(3)
        c.random.seed(4)
        s0 = _native.mt_spec_stats()
        off = [device_shares(c, sec, N, 5) for _ in range(4)]
        assert delta(s0, _native.mt_spec_stats())["launched"] == 0
    assert all(torch.equal(x, y) for x, y in zip(on, off))
    assert a.random.getstate() == c.random.getstate()
    small = (1 << 22) - 1  # 2^23 - 2 coefficients
    s0 = _native.mt_spec_stats()
    for _ in range(3):
        device_shares(a, sec[:small], small, 5)
    assert delta(s0, _native.mt_spec_stats())["launched"] == 0


@pytest.mark.parametrize("n,tm1,pre", [(2561, 2, 0), (2561, 2, 623), (2048 * 5 + 1, 1, 300), (400, 2, 17),
                                       (5 * 1024 + 18, 1, 600), ((1 << 20) + 1, 2, 5), (1 << 23, 2, 0),
                                       ((1 << 23) + 7, 2, 611)])
@pytest.mark.parametrize("tail", ["1", "0"])
def test_final_state_by_the_last_substream(n, tm1, pre, tail, monkeypatch):
    """CPython's final state comes from the last substream's tail (DN_MT_TAIL_FIN,
    the product default) or, in the tuning build with DN_MT_TAIL_FIN=0, from a
    final-state wave: both equal the host draw's block and final state — with
    a last substream of 1 .. 18 draws (the final array then starts in the
    substream's window, before its first output), a single substream starting
    inside the caller's array, and the 2^24-scale draws."""
    a = random.Random(n * 5 + tm1 + pre)
    a.getrandbits(32 * pre)
    b = random.Random()
    b.setstate(a.getstate())
    want = torch.from_numpy(_native.mt_draw_coeffs(a, n, tm1)).to(dev())
    got = torch.zeros((tm1, field.vec_bytes(n)), dtype=torch.uint8, device=dev())
    if tail == "0":
        monkeypatch.setenv("DN_MT_TAIL_FIN", "0")
        with _native.library(_native.TUNING_LIB):
            assert _native.mt_draw_coeffs_device(b, n, tm1, got)
    else:
        assert _native.mt_draw_coeffs_device(b, n, tm1, got)
    assert torch.equal(got, want)
    assert a.getstate() == b.getstate()


@pytest.mark.parametrize("cb", ["2", "3"])
@pytest.mark.parametrize("n,tm1,pre", [(1 << 23, 2, 0), ((1 << 24) + 1, 1, 333), ((1 << 22) + 1000, 4, 7)])
def test_two_bit_jump_kernel_equals_host_draw(n, tm1, pre, cb, monkeypatch):
    """mt_jumpc_kernel<4, CB> (2-bit chunks in an 11 KB table, or 3-bit chunks
    with bit 0 alone in a 19.3 KB table without T[0]; four waves per
    workgroup: the kernels that fit beside the generation) computing the
    2^24-scale draw's direct level in place of mt_jump_kernel (tuning build,
    DN_MT_SPEC_PROBE=5, DN_MT_BESIDE_CB): the host draw's block and final state."""
    monkeypatch.setenv("DN_MT_BESIDE_CB", cb)
    a = random.Random(n + tm1 + pre)
    a.getrandbits(32 * pre)
    b = random.Random()
    b.setstate(a.getstate())
    want = torch.from_numpy(_native.mt_draw_coeffs(a, n, tm1)).to(dev())
    got = torch.zeros((tm1, field.vec_bytes(n)), dtype=torch.uint8, device=dev())
    monkeypatch.setenv("DN_MT_SPEC_PROBE", "5")
    with _native.library(_native.TUNING_LIB):
        assert _native.mt_draw_coeffs_device(b, n, tm1, got)
    assert torch.equal(got, want)
    assert a.getstate() == b.getstate()


def test_loop_without_beside_levels(monkeypatch):
    """The 2^24-scale speculation with the beside chain off (tuning build,
    DN_MT_SPEC_BESIDE=0: the next call's W_idx from the last substream, its
    level after the generation): hits, and the host draw's shares and state."""
    monkeypatch.setenv("DN_MT_SPEC_BESIDE", "0")
    with _native.library(_native.TUNING_LIB):
        _loop_case((1 << 23) + 9, 3, 5, 100)


@pytest.mark.parametrize("parts", ["4", "8"])
def test_four_bit_contiguous_jump_kernel_equals_host_draw(parts, monkeypatch):
    """mt_jumpc_kernel<16, 4> (4-bit chunks, the 45 KB contiguous table, two
    workgroups per CU) computing the 2^24-scale direct level in place of
    mt_jump_kernel (tuning build: DN_MT_JUMP4B=1, DN_MT_PARTS_B parts per
    jump): the host draw's block and final state."""
    n, tm1 = (1 << 23) + 5, 2
    a = random.Random(int(parts))
    a.getrandbits(32 * 77)
    b = random.Random()
    b.setstate(a.getstate())
    want = torch.from_numpy(_native.mt_draw_coeffs(a, n, tm1)).to(dev())
    got = torch.zeros((tm1, field.vec_bytes(n)), dtype=torch.uint8, device=dev())
    monkeypatch.setenv("DN_MT_JUMP4B", "1")
    monkeypatch.setenv("DN_MT_PARTS_B", parts)
    monkeypatch.setenv("DN_MT_SPEC", "0")
    with _native.library(_native.TUNING_LIB):
        assert _native.mt_draw_coeffs_device(b, n, tm1, got)
    assert torch.equal(got, want)
    assert a.getstate() == b.getstate()


def test_speculation_under_threads_and_interleaved_objects():
    """Two threads, each looping over the 2^24-scale draw with its own
    SecretShare (the device's speculation state is taken by try_lock: a call
    finding it busy runs unspeculated), then two objects interleaved on one
    thread (each call misses the other's speculation): every call equals the
    host draw + split, with the same final states."""
    import threading

    N = (1 << 23) + 3
    sec = torch.from_numpy(secrets_int64(12, N)).to(dev())
    res, err = {}, []

    def run(i):
        try:
            torch.cuda.set_device(dev())
            ss = shamir.SecretShare(3)
            ss.random.seed(500 + i)
            outs = [device_shares(ss, sec, N, 5) for _ in range(4)]
            torch.cuda.synchronize()
            res[i] = (outs, ss.random.getstate())
        except Exception as e:  # surfaced below
            err.append(e)

    ths = [threading.Thread(target=run, args=(i,)) for i in range(2)]
    for th in ths:
        th.start()
    for th in ths:
        th.join()
    assert not err, err
    for i in range(2):
        ref = shamir.SecretShare(3)
        ref.random.seed(500 + i)
        for got in res[i][0]:
            assert torch.equal(got, host_shares(ref.random, sec, N, 3, 5))
        assert ref.random.getstate() == res[i][1]
    a, b, ra, rb = shamir.SecretShare(3), shamir.SecretShare(3), shamir.SecretShare(3), shamir.SecretShare(3)
    for x, y in ((a, ra), (b, rb)):
        x.random.seed(id(x) % 1000)
        y.random.setstate(x.random.getstate())
    for x, y in ((a, ra), (a, ra), (b, rb), (a, ra), (b, rb), (b, rb)):
        assert torch.equal(device_shares(x, sec, N, 5), host_shares(y.random, sec, N, 3, 5))
        assert x.random.getstate() == y.random.getstate()
