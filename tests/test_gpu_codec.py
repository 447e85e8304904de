"""HIP share wire codec vs the reference's bytes.

The packed records must equal, byte for byte, the `_share_to_bytes` output
the reference produced for the same shares (tests/golden f1/f2/f3, generated
from delta_node/crypto/shamir/shamir.py), and decoding must give back the
share vectors.  Larger and edge-case vectors are checked against a host
encoding with the reference's own codec restated (oracle/py_shamir.py).
"""
import random

import numpy as np
import pytest
import torch

from delta_node.crypto import shamir
from delta_node.crypto.shamir import codec, field
from golden.fixtures import P, load_json, load_npz, manifest, unpack_share_bytes
from oracle.py_shamir import share_to_bytes

pytestmark = pytest.mark.gpu


def dev():
    return torch.device("cuda", torch.cuda.current_device())


@pytest.mark.parametrize("key", ["f1", "f2"])
def test_encode_matches_reference_share_bytes(key):
    cfg = manifest()[key]
    z = load_npz(cfg["file"])
    N, n, t = cfg["N"], cfg["n"], cfg["t"]
    ss = shamir.SecretShare(t)
    ss.random.seed(cfg["mt_seed"])
    block = ss.make_shares_vec(torch.from_numpy(z["secrets"]), n)
    for x in range(1, n + 1):
        packed, offs = codec.encode_share_vec(block[x - 1], N, x)
        recs = codec.records_to_list(packed.cpu(), offs.cpu())
        want = [unpack_share_bytes(z["share_bytes"], z["share_offsets"], e * n + x - 1) for e in range(N)]
        assert recs == want, x
        assert bytes(packed.cpu().numpy()) == b"".join(want)
        vec, xs = codec.decode_share_vec(packed, offs, N)
        assert torch.equal(vec[: field.vec_bytes(N)], block[x - 1]) or np.array_equal(
            field.vec_to_limbs(vec.cpu().numpy(), N), field.vec_to_limbs(block[x - 1].cpu().numpy(), N))
        assert torch.all(xs == x)


def test_encode_edge_values_and_wide_x():
    vals = [0, 1, 255, 256, 2**64 - 1, 2**512, P - 1, 2**520, 2**519 + 5, 7 << 300] + \
        [random.Random(i).randrange(P) for i in range(300)]
    n = len(vals)
    vec = torch.from_numpy(field.ints_to_vec(vals)).to(dev())
    for x in (1, 5, 255, 256, 300, 65535, 2**40 + 3):
        packed, offs = codec.encode_share_vec(vec, n, x)
        recs = codec.records_to_list(packed.cpu(), offs.cpu())
        assert recs == [share_to_bytes(x, y) for y in vals], x
        back, xs = codec.decode_share_vec(packed, offs, n)
        assert field.vec_to_ints(back.cpu().numpy(), n) == vals
        assert torch.all(xs == x)


@pytest.mark.parametrize("n", [1, 255, 1023, 1024, 1025, 70001])
def test_encode_ragged_random_vs_host(n):
    rng = random.Random(n)
    vals = [rng.randrange(P) >> rng.randrange(0, 521) for _ in range(n)]  # many byte lengths
    vec = torch.from_numpy(field.ints_to_vec(vals)).to(dev())
    packed, offs = codec.encode_share_vec(vec, n, 3)
    want = b"".join(share_to_bytes(3, y) for y in vals)
    assert bytes(packed.cpu().numpy()) == want
    assert int(offs[n].item()) == len(want)
    back, _ = codec.decode_share_vec(packed, offs, n)
    assert field.vec_to_ints(back.cpu().numpy(), n) == vals


def test_decode_reduces_like_resolve_and_flags_oversize():
    """Records as a peer might send them: leading zero bytes, y >= p (reduced
    mod p as resolve_shares does, shamir.py:86-88), oversize y (flagged)."""
    ys = [0, 5, P, P + 9, (1 << 527) + 1]
    recs = [bytes([1, 2]) + b"\x00\x00" + (5).to_bytes(1, "big")] + \
           [share_to_bytes(2, y) for y in ys]
    packed = torch.tensor(list(b"".join(recs)), dtype=torch.uint8, device=dev())
    offs = torch.tensor(np.cumsum([0] + [len(r) for r in recs]), dtype=torch.int64, device=dev())
    vec, xs = codec.decode_share_vec(packed, offs, len(recs))
    assert field.vec_to_ints(vec.cpu().numpy(), len(recs)) == [5] + [y % P for y in ys]
    bad = torch.tensor(list(share_to_bytes(2, 1 << 560)), dtype=torch.uint8, device=dev())
    with pytest.raises(ValueError):
        codec.decode_share_vec(bad, torch.tensor([0, bad.numel()], dtype=torch.int64, device=dev()), 1)


def test_caller_buffers_and_deferred_bad_check():
    """encode / decode into caller buffers (no allocation),
    the decoder's bad-record count added to a caller flag without a sync per
    call and checked once (codec.check_bad) — same bytes as the allocating form."""
    n = 5000
    rng = random.Random(7)
    vals = [rng.randrange(P) >> rng.randrange(0, 521) for _ in range(n)]
    vec = torch.from_numpy(field.ints_to_vec(vals)).to(dev())
    want_p, want_o = codec.encode_share_vec(vec, n, 3)
    out = torch.empty(codec.encoded_capacity(n, 3), dtype=torch.uint8, device=dev())
    offs = torch.empty(n + 1, dtype=torch.int64, device=dev())
    p2, o2 = codec.encode_share_vec(vec, n, 3, out=out, offsets=offs)
    assert p2.data_ptr() == out.data_ptr() and torch.equal(p2, want_p) and torch.equal(o2, want_o)
    dv = torch.empty(field.vec_bytes(n), dtype=torch.uint8, device=dev())
    dx = torch.empty(n, dtype=torch.int64, device=dev())
    flag = torch.zeros(1, dtype=torch.int32, device=dev())
    for _ in range(3):
        v2, x2 = codec.decode_share_vec(want_p, want_o, n, out=dv, xs=dx, bad=flag)
    codec.check_bad(flag)
    assert v2.data_ptr() == dv.data_ptr() and field.vec_to_ints(dv.cpu().numpy(), n) == vals
    assert torch.all(x2 == 3)
    bad = torch.tensor(list(share_to_bytes(2, 1 << 560)), dtype=torch.uint8, device=dev())
    bo = torch.tensor([0, bad.numel()], dtype=torch.int64, device=dev())
    codec.decode_share_vec(bad, bo, 1, bad=flag)
    codec.decode_share_vec(bad, bo, 1, bad=flag)
    assert int(flag.item()) == 2  # added to, not overwritten
    with pytest.raises(ValueError, match="2 records"):
        codec.check_bad(flag)
    with pytest.raises(ValueError):
        codec.decode_share_vec(want_p, want_o, n, out=dv[:10])
    with pytest.raises(ValueError):
        codec.decode_share_vec(want_p, want_o, n, bad=torch.zeros(1, dtype=torch.int64, device=dev()))


def test_byte_api_fixture_through_vector_codec():
    """f3 edge cases: each case's shares, re-encoded from one-element vectors, equal the reference bytes."""
    f3 = load_json("f3_edge.json")
    for case in f3["cases"][:60]:
        ys = [int.from_bytes(bytes.fromhex(s)[1 + bytes.fromhex(s)[0]:], "big") for s in case["shares"]]
        vec = torch.from_numpy(field.ints_to_vec(ys)).to(dev())
        for x in (1, len(ys)):
            packed, offs = codec.encode_share_vec(vec, len(ys), x)
            recs = codec.records_to_list(packed.cpu(), offs.cpu())
            assert recs[x - 1] == bytes.fromhex(case["shares"][x - 1])


def test_decode_wide_windows_and_untrusted_offsets():
    """Wave windows of records padded with leading zero bytes (larger than the
    LDS slice: byte-serial path) beside normal ones, a 69-byte y with one
    leading zero and 68 significant bytes, and offsets a peer got wrong
    (decreasing / out of range: flagged, never read outside the input)."""
    rng = random.Random(11)
    ys = [rng.randrange(1 << 544) for _ in range(300)]
    recs = []
    for i, y in enumerate(ys):
        yb = y.to_bytes((y.bit_length() + 7) // 8, "big")
        pad = 100 if 64 <= i < 128 else (1 if i % 7 == 0 else 0)
        recs.append(bytes([1, 4]) + b"\x00" * pad + yb)
    packed = torch.tensor(list(b"".join(recs)), dtype=torch.uint8, device=dev())
    offs = torch.tensor(np.cumsum([0] + [len(r) for r in recs]), dtype=torch.int64, device=dev())
    vec, xs = codec.decode_share_vec(packed, offs, len(recs))
    assert field.vec_to_ints(vec.cpu().numpy(), len(recs)) == [y % P for y in ys]
    assert torch.equal(xs.cpu(), torch.full((len(recs),), 4, dtype=torch.int64))
    bad_offs = offs.clone()
    bad_offs[10] = bad_offs[12] + 5  # record 10 runs past record 11's start, record 11 goes backwards
    with pytest.raises(ValueError):
        codec.decode_share_vec(packed, bad_offs, len(recs))
    far = offs.clone()
    far[-1] = far[-1] + (1 << 40)  # last record claims bytes far past the input
    with pytest.raises(ValueError):
        codec.decode_share_vec(packed, far, len(recs))


@pytest.mark.parametrize("shift", [4, 8, 12])
def test_unaligned_buffers_take_the_narrow_path(shift):
    """Buffers not 16-B aligned (a 4-B-aligned slice of a larger allocation)
    take the 4-B staging / store path of the codec kernels; results equal the
    aligned (16-B) path byte for byte."""
    import ctypes

    L = codec._lib()
    N = 5000 + shift
    vals = [random.Random(shift * 100003 + i).randrange(P) for i in range(N)]
    vec = torch.from_numpy(field.ints_to_vec(vals)).to(dev())
    want_packed, want_offs = codec.encode_share_vec(vec, N, 3)
    cap = int(L.dn_m521_encoded_capacity(N, 3))
    big = torch.zeros(cap + 64, dtype=torch.uint8, device=dev())
    out = big[shift:]  # data_ptr % 16 == shift
    assert out.data_ptr() % 16 == shift
    offs = torch.empty(N + 1, dtype=torch.int64, device=dev())
    sb = int(L.dn_m521_codec_scratch_bytes(N))
    scratch = torch.empty(sb, dtype=torch.uint8, device=dev())
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    assert L.dn_m521_encode_shares(vec.data_ptr(), N, 3, offs.data_ptr(), out.data_ptr(), cap, scratch.data_ptr(), sb,
                                   st) == 0
    total = int(want_offs[N].item())
    assert torch.equal(offs, want_offs)
    assert torch.equal(out[:total], want_packed)
    # decode from the unaligned copy
    back = torch.empty(field.vec_bytes(N), dtype=torch.uint8, device=dev())
    xs = torch.empty(N, dtype=torch.int64, device=dev())
    bad = torch.zeros(1, dtype=torch.int32, device=dev())
    assert L.dn_m521_decode_shares(out.data_ptr(), total, offs.data_ptr(), N, back.data_ptr(), xs.data_ptr(),
                                   bad.data_ptr(), st) == 0
    torch.cuda.synchronize()
    assert int(bad.item()) == 0
    assert field.vec_to_ints(back.cpu().numpy(), N) == vals
    assert torch.all(xs == 3)
