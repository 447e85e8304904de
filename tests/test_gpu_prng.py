"""dn_m521_split_prng / dn_m521_prng_coeffs (SURVEY.md §8(b), §8(d) config 2'):
device-generated coefficients vs the C restatement (oracle/chacha_oracle.c,
itself pinned to OpenSSL's ChaCha20 in tests/test_prng_oracle.py), and the
split that consumes them vs the split of the same coefficients read from
memory and vs the C oracle.  All comparisons bit-exact."""
import numpy as np
import pytest
import torch

from delta_node.crypto import shamir
from delta_node.crypto.shamir import _native, field
from golden.fixtures import P, secrets_int64
from oracle import c_oracle

pytestmark = pytest.mark.gpu
KEY = bytes((11 * i + 7) & 0xFF for i in range(32))


def dev():
    return torch.device("cuda", torch.cuda.current_device())


def coeff_block(N, tm1, key=KEY, nonce=5, rounds=20, off=0):
    co = torch.empty((tm1, field.vec_bytes(N)), dtype=torch.uint8, device=dev())
    _native.prng_coeffs(key, nonce, rounds, off, co, N, tm1)
    return co


def block_limbs(block, n):
    h = block.cpu().numpy()
    return np.stack([field.vec_to_limbs(h[s], n) for s in range(h.shape[0])])


@pytest.mark.parametrize("N", [1, 255, 256, 1000, 4099])
@pytest.mark.parametrize("t", [2, 3, 5, 8])
@pytest.mark.parametrize("rounds,off", [(20, 0), (12, 512), (8, 256 * 1001)])
def test_prng_coeffs_match_oracle(N, t, rounds, off):
    co = coeff_block(N, t - 1, rounds=rounds, off=off)
    want = c_oracle.prng_coeffs(KEY, 5, off, N, t - 1, rounds=rounds)  # [N, t-1, 17]
    assert np.array_equal(block_limbs(co, N), want.transpose(1, 0, 2))


@pytest.mark.parametrize("N", [1, 257, 3000])
@pytest.mark.parametrize("t,n", [(2, 3), (3, 5), (5, 9), (8, 8), (4, 300)])
def test_split_prng_equals_split_of_materialized_coeffs(N, t, n):
    sec = torch.from_numpy(secrets_int64(N + t, N)).to(dev())
    shares = torch.empty((n, field.vec_bytes(N)), dtype=torch.uint8, device=dev())
    _native.split_prng(sec, KEY, 5, 20, 0, shares, N, t, n)
    co = coeff_block(N, t - 1)
    ref = torch.empty_like(shares)
    _native.split_u64(sec, co, ref, N, t, n)
    assert np.array_equal(block_limbs(shares, N), block_limbs(ref, N))  # valid elements (tile tails unwritten)
    want = c_oracle.split(sec.cpu().numpy(), c_oracle.prng_coeffs(KEY, 5, 0, N, t - 1), t, n)
    assert np.array_equal(block_limbs(shares, N), want)


def test_split_prng_sharded_equals_unsharded():
    N, t, n = 256 * 37 + 11, 3, 5
    sec = torch.from_numpy(secrets_int64(3, N)).to(dev())
    whole = torch.empty((n, field.vec_bytes(N)), dtype=torch.uint8, device=dev())
    _native.split_prng(sec, KEY, 9, 20, 0, whole, N, t, n)
    cut = 256 * 20
    for lo, hi in ((0, cut), (cut, N)):
        part = torch.empty((n, field.vec_bytes(hi - lo)), dtype=torch.uint8, device=dev())
        _native.split_prng(sec[lo:hi].contiguous(), KEY, 9, 20, lo, part, hi - lo, t, n)
        got = block_limbs(part, hi - lo)
        assert np.array_equal(got, block_limbs(whole, N)[:, lo:hi])


def test_make_shares_vec_prng_roundtrip_and_key():
    N = (1 << 20) + 3
    vals = torch.from_numpy(secrets_int64(8, N))
    ss = shamir.SecretShare(3)
    block, key = ss.make_shares_vec_prng(vals, 5)
    assert len(key) == 32
    for xs in ([1, 2, 3], [1, 3, 5], [2, 4, 5]):
        back = ss.resolve_shares_vec([block[x - 1] for x in xs], xs, N)
        assert torch.equal(back.cpu(), vals)
    again, _ = ss.make_shares_vec_prng(vals, 5, key=key)
    assert np.array_equal(block_limbs(again[:, : field.vec_bytes(4096)], 4096),
                          block_limbs(block[:, : field.vec_bytes(4096)], 4096))
    assert torch.equal(ss.resolve_shares_vec([again[0], again[1], again[3]], [1, 2, 4], N).cpu(), vals)
    other, _ = ss.make_shares_vec_prng(vals, 5, key=key, nonce=1)
    assert not torch.equal(other[1, :4096], block[1, :4096])
    # coefficients are in [1, p-1] (spot check through the materialized stream)
    lim = block_limbs(coeff_block(4096, 2, key=key, nonce=0), 4096)
    ints = [sum(int(w) << (32 * k) for k, w in enumerate(lim[j, e])) for j in range(2) for e in range(0, 4096, 97)]
    assert all(1 <= v <= P - 1 for v in ints)


def test_split_prng_argument_errors():
    sec = torch.zeros(256, dtype=torch.int64, device=dev())
    sh = torch.empty((5, field.vec_bytes(256)), dtype=torch.uint8, device=dev())
    with pytest.raises(ValueError):
        _native.split_prng(sec, KEY, 0, 10, 0, sh, 256, 3, 5)  # rounds
    with pytest.raises(ValueError):
        _native.split_prng(sec, KEY, 0, 20, 100, sh, 256, 3, 5)  # unaligned offset
    with pytest.raises(NotImplementedError):
        _native.split_prng(sec, KEY, 0, 20, 0, sh, 256, 9, 9)  # t > 8
    with pytest.raises(ValueError):
        _native.split_prng(sec, KEY, 0, 20, 0, sh, 256, 6, 5)  # t > n
    with pytest.raises(ValueError):
        _native.split_prng(sec, KEY[:16], 0, 20, 0, sh, 256, 3, 5)
