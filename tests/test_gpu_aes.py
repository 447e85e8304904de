"""The share envelope on the GPU (csrc/aes_envelope.hip, SURVEY.md §8(f) row 2,
second half) against the reference's layers.

Expected text for (key, nonce, data): base64.b64encode(nonce + ct) — the
reference's aes.encrypt (crypto/aes/aes.py:8-14) with its cipher restated in
oracle/aes_oracle.c (pinned to OpenSSL and the NIST vectors in
test_aes_oracle.py) — and "0x" + its .hex() for the JSON form
(serialize.bytes_to_hex, runner/horizontal/commu.py:23-49).  Decryption is
checked against bytes.fromhex / base64.b64decode, including their errors.
Bit-exact throughout.
"""
import base64
import binascii

import numpy as np
import pytest
import torch

from delta_node.crypto import aes, shamir
from delta_node.crypto.shamir import _native, codec
from golden.fixtures import secrets_int64
from oracle import c_oracle

pytestmark = pytest.mark.gpu

KEYS = [bytes(range(32)), bytes(range(100, 116)), bytes(range(7, 31))]
NONCES = [bytes(16), b"\xff" * 16, b"\xff" * 15 + b"\xfd", bytes(8) + b"\xff" * 8, bytes(range(200, 216))]
SIZES = [0, 1, 2, 15, 16, 17, 31, 32, 33, 47, 48, 49, 63, 64, 65, 79, 80, 81, 95, 96, 97, 127, 128, 129,
         191, 192, 1000, 3071, 3072, 3073, 6128, 6129, 12345, 98288]


def dev():
    return torch.device("cuda", torch.cuda.current_device())


def to_dev(b: bytes, skew: int = 0):
    """b on the device, starting `skew` bytes into a fresh (aligned) allocation."""
    buf = torch.zeros(len(b) + skew + 16, dtype=torch.uint8, device=dev())
    if b:
        buf[skew:skew + len(b)] = torch.frombuffer(bytearray(b), dtype=torch.uint8).to(dev())
    return buf[skew:skew + len(b)]


def host(t) -> bytes:
    return bytes(t.cpu().numpy())


def rand_bytes(n: int, seed: int) -> bytes:
    return np.random.default_rng(seed).integers(0, 256, n, dtype=np.uint8).tobytes()


def want_text(key, nonce, data, hex_=False) -> bytes:
    b = base64.b64encode(nonce + c_oracle.aes_ctr(key, nonce, data))
    return b"0x" + b.hex().encode() if hex_ else b


def ref_decrypt(key, text: bytes, hex_=False) -> bytes:
    """The receiver's path: hex_to_bytes (hex.py:29-41) then aes.decrypt (aes.py:17-23)."""
    if hex_:
        s = text.decode("ascii")
        text = bytes.fromhex(s[2:] if s.startswith("0x") else s)
    raw = base64.b64decode(text)
    if len(raw[:16]) != 16:
        raise ValueError("Invalid nonce size")
    return c_oracle.aes_ctr(key, raw[:16], raw[16:])


@pytest.mark.parametrize("n", SIZES)
def test_encrypt_matches_reference_layers(n):
    data = rand_bytes(n, n)
    for key in KEYS:
        for nonce in NONCES[:3]:
            for hex_ in (False, True):
                got = host(aes.encrypt_vec(key, to_dev(data), nonce=nonce, hex=hex_))
                assert got == want_text(key, nonce, data, hex_), (len(key), nonce.hex(), hex_)


@pytest.mark.parametrize("n", SIZES)
def test_decrypt_forms(n):
    data = rand_bytes(n, 1000 + n)
    key, nonce = KEYS[0], NONCES[4]
    assert host(aes.decrypt_vec(key, to_dev(want_text(key, nonce, data)))) == data
    hx = want_text(key, nonce, data, True)
    assert host(aes.decrypt_vec(key, to_dev(hx), hex=True)) == data
    assert host(aes.decrypt_vec(key, to_dev(hx[2:]), hex=True)) == data  # without "0x"
    assert host(aes.decrypt_vec(key, to_dev(b"0x" + hx[2:].upper()), hex=True)) == data  # coord.py:93 allows A-F


@pytest.mark.parametrize("ntab", ["4", "2"])
def test_table_layouts_and_ctr(ntab, monkeypatch):
    """Both T-table layouts (tuning build's DN_AES_TABLES) give the oracle's bytes."""
    monkeypatch.setenv("DN_AES_TABLES", ntab)
    data = rand_bytes(5000, 3)
    with _native.library(_native.TUNING_LIB):
        for key in KEYS:
            for nonce in NONCES:
                assert host(aes.ctr_vec(key, nonce, to_dev(data))) == c_oracle.aes_ctr(key, nonce, data)
                text = want_text(key, nonce, data, True)
                assert host(aes.encrypt_vec(key, to_dev(data), nonce=nonce, hex=True)) == text
                assert host(aes.decrypt_vec(key, to_dev(text), hex=True)) == data


@pytest.mark.parametrize("skew", [1, 2, 3, 4, 5, 7, 8, 9, 13, 15])
def test_inputs_at_any_byte_offset(skew):
    data = rand_bytes(4099, skew)
    key, nonce = KEYS[0], NONCES[3]
    hx, b64 = want_text(key, nonce, data, True), want_text(key, nonce, data)
    assert host(aes.encrypt_vec(key, to_dev(data, skew), nonce=nonce, hex=True)) == hx
    assert host(aes.encrypt_vec(key, to_dev(data, skew), nonce=nonce)) == b64
    assert host(aes.decrypt_vec(key, to_dev(hx, skew), hex=True)) == data
    assert host(aes.decrypt_vec(key, to_dev(b64, skew))) == data
    assert host(aes.ctr_vec(key, nonce, to_dev(data, skew))) == c_oracle.aes_ctr(key, nonce, data)


def _odd_texts(b64: bytes):
    yield b64[:40] + b"\n" + b64[40:]   # b64decode drops characters outside the alphabet
    yield b64.rstrip(b"=")              # missing padding
    yield b64[:8] + b"=" + b64[9:]      # '=' inside
    yield b64[:-4] + b"QQ=="            # another canonical tail
    yield b64[:10] + b"*" + b64[11:]
    yield base64.b64encode(b"short nonce")
    yield b""
    yield b"===="


def test_noncanonical_text_behaves_like_reference():
    key, nonce = KEYS[0], NONCES[4]
    for n in (0, 5, 100):
        data = rand_bytes(n, n)
        for text in _odd_texts(want_text(key, nonce, data)):
            for hex_ in (False, True):
                t = (b"0x" + text.hex().encode()) if hex_ else text
                try:
                    want = ref_decrypt(key, t, hex_)
                except ValueError as e:  # binascii.Error is a ValueError
                    with pytest.raises(type(e)):
                        aes.decrypt_vec(key, to_dev(t), hex=hex_)
                    continue
                assert host(aes.decrypt_vec(key, to_dev(t), hex=hex_)) == want, (n, t[:60])
    data = rand_bytes(300, 9)
    hx = want_text(key, nonce, data, True)[2:].decode()
    spaced = "0x" + " ".join(hx[i:i + 2] for i in range(0, len(hx), 2))  # bytes.fromhex skips the spaces
    assert host(aes.decrypt_vec(key, to_dev(spaced.encode()), hex=True)) == data
    with pytest.raises(ValueError):
        aes.decrypt_vec(key, to_dev(b"0xzz" + hx[2:].encode()), hex=True)
    with pytest.raises(binascii.Error):
        aes.decrypt(key, want_text(key, nonce, data)[:-1])


def test_bytes_api():
    key = KEYS[0]
    for data in (b"", b"x", b"delta-node seed share", bytes(range(256)) * 3):
        s = aes.encrypt(key, data)
        raw = base64.b64decode(s)
        assert len(raw) == 16 + len(data) and raw[16:] == c_oracle.aes_ctr(key, raw[:16], data)
        assert aes.decrypt(key, s) == data
        assert aes.decrypt(key, s.decode()) == data
        assert aes.encrypt(key, data, nonce=NONCES[1]) == want_text(key, NONCES[1], data)
    assert aes.encrypt(key, b"abc") != aes.encrypt(key, b"abc")  # os.urandom nonce, as the reference


@pytest.mark.parametrize("n", [0, 1, 33, 68, 100, 4099, 70000])
def test_host_and_device_agree(n, monkeypatch):
    """The byte API's host cipher (csrc/host_aes.cpp) and the device kernels give
    the same text at a fixed nonce, and each opens the other's; above
    HOST_MAX_BYTES the byte API takes the device path (same bytes)."""
    from delta_node.crypto.aes import aes as aes_mod

    data = rand_bytes(n, 50 + n)
    for key in KEYS:
        for nonce in NONCES:
            text = aes.encrypt(key, data, nonce=nonce)  # host (n <= HOST_MAX_BYTES)
            assert text == host(aes.encrypt_vec(key, to_dev(data), nonce=nonce))
            assert host(aes.decrypt_vec(key, to_dev(text))) == data
            assert aes.decrypt(key, text) == data
            assert aes.ctr_host(key, nonce, data) == host(aes.ctr_vec(key, nonce, to_dev(data)))
    monkeypatch.setattr(aes_mod, "HOST_MAX_BYTES", 0)  # every byte message through the GPU
    text = aes.encrypt(KEYS[0], data, nonce=NONCES[3])
    assert text == want_text(KEYS[0], NONCES[3], data)
    assert aes.decrypt(KEYS[0], text) == data


def test_encrypt_into_a_reused_buffer():
    """encrypt_vec(..., out=encrypt_buffer(n, hex)): the same text as the
    allocating call, written into the caller's buffer."""
    key = KEYS[0]
    for n in (0, 1, 47, 4099):
        data = to_dev(rand_bytes(n, n + 3))
        for hex_ in (False, True):
            buf = aes.encrypt_buffer(n, hex_, dev())
            for nonce in NONCES[:2]:
                got = aes.encrypt_vec(key, data, nonce=nonce, hex=hex_, out=buf)
                assert host(got) == want_text(key, nonce, host(data), hex_)
                assert buf.data_ptr() <= got.data_ptr() < buf.data_ptr() + buf.numel()
    with pytest.raises(ValueError):
        aes.encrypt_vec(key, to_dev(b"x" * 100), hex=True, out=aes.encrypt_buffer(10, True, dev()))


def test_large_message_sampled_against_oracle():
    n = (1 << 26) + 77
    g = torch.Generator(device=dev())
    g.manual_seed(5)
    data = torch.randint(0, 256, (n,), dtype=torch.uint8, device=dev(), generator=g)
    key, nonce = KEYS[0], bytes(8) + b"\xff" * 7 + b"\xf0"  # the low 64 counter bits wrap inside the message
    text = aes.encrypt_vec(key, data, nonce=nonce, hex=True)
    b64_len = len(base64.b64encode(bytes(16 + n)))
    assert text.numel() == 2 + 2 * b64_len
    assert torch.equal(aes.decrypt_vec(key, text, hex=True), data)
    units = (b64_len + 63) // 64
    for u in (0, 1, 12345, units - 5):  # windows of 4 units, decoded on the host
        t = host(text[2 + 128 * u: 2 + 128 * (u + 4)])
        m = base64.b64decode(bytes.fromhex(t.decode()))  # message bytes [48u, ...)
        start = 48 * u - 16
        if u == 0:
            assert m[:16] == nonce
            m, start = m[16:], 0
        iv = ((int.from_bytes(nonce, "big") + start // 16) % (1 << 128)).to_bytes(16, "big")
        assert m == c_oracle.aes_ctr(key, iv, host(data[start:start + len(m)])), u


def test_vector_share_envelope_roundtrip():
    """make_shares_vec -> share records (codec) -> sealed JSON text -> back."""
    N, key, nonce = 3000, KEYS[0], NONCES[4]
    ss = shamir.SecretShare(3)
    ss.random.seed(21)
    # zeroed: the lanes past N of the last tile are never written (nor compared below)
    block = torch.zeros((5, _native.vec_bytes(N)), dtype=torch.uint8, device=dev())
    ss.make_shares_vec(torch.from_numpy(secrets_int64(4, N)), 5, out=block)
    packed, offs = codec.encode_share_vec(block[1], N, 2)
    env = aes.encrypt_vec(key, packed, nonce=nonce, hex=True)
    assert host(env) == want_text(key, nonce, host(packed), True)
    recs = aes.decrypt_vec(key, env, hex=True)
    vec, xs = codec.decode_share_vec(recs, offs, N)
    assert torch.equal(vec, block[1]) and bool((xs == 2).all())


def test_bad_characters_inside_full_waves():
    """A bad character in the middle of a long text — where the decrypt reads
    whole waves of units line by line (decrypt_fused_kernel) — is flagged, and
    the call then behaves as the reference's own calls do (aes.py:17-23,
    hex.py:29-41)."""
    key, nonce = KEYS[0], NONCES[2]
    data = rand_bytes(300_000, 77)
    b64 = want_text(key, nonce, data)
    mid = len(b64) // 2 + 5
    for bad in (b"*", b"=", b"\n", b"-"):
        t64 = b64[:mid] + bad + b64[mid + 1:]
        for hex_ in (False, True):
            t = (b"0x" + t64.hex().encode()) if hex_ else t64
            try:
                want = ref_decrypt(key, t, hex_)
            except ValueError as e:
                with pytest.raises(type(e)):
                    aes.decrypt_vec(key, to_dev(t), hex=hex_)
                continue
            assert host(aes.decrypt_vec(key, to_dev(t), hex=hex_)) == want, (bad, hex_)
    hx = want_text(key, nonce, data, True)
    for bad in (b"g", b" ", b"\x80"):
        t = hx[:2 + 2 * mid] + bad + hx[3 + 2 * mid:]
        try:
            want = ref_decrypt(key, t, True)
        except ValueError:  # fromhex / the ascii decode refuse it
            with pytest.raises(ValueError):
                aes.decrypt_vec(key, to_dev(t), hex=True)
            continue
        assert host(aes.decrypt_vec(key, to_dev(t), hex=True)) == want, bad
