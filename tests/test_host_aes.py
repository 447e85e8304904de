"""The share envelope's byte API on the host (csrc/host_aes.cpp): `aes.encrypt`
/ `aes.decrypt` (reference delta_node/crypto/aes/aes.py:8-23), called once per
~70-byte share by the runner (runner/horizontal/agg.py:192-196, :258, :265).

Checked against the same independent vectors as the oracle (FIPS-197
Appendix C, SP 800-38A F.5.1 / F.5.5, the 252 `openssl enc -aes-*-ctr`
outputs of tests/golden/aes_kat.json) and the C oracle, with both host ciphers
(AES-NI and the T-table fallback, the tuning build's DN_AES_HOST=table), plus
the reference's parse and errors for text that is not canonical base64, and
the per-call latency (<= 10 us for 68- and 33-byte payloads).  No GPU: the
device-vs-host comparison is tests/test_gpu_aes.py::test_host_and_device_agree.
"""
import base64
import binascii
import ctypes
import os
import time

import numpy as np
import pytest

from delta_node.crypto import aes
from delta_node.crypto.aes import aes as aes_mod
from delta_node.crypto.shamir import _native
from golden.fixtures import load_json
from oracle import c_oracle
from test_aes_oracle import FIPS197, PT, SP800, SP800_IV, SP800_PT

KEYS = [bytes(range(32)), bytes(range(100, 116)), bytes(range(7, 31))]
NONCES = [bytes(16), b"\xff" * 16, b"\xff" * 15 + b"\xfd", bytes(8) + b"\xff" * 8, bytes(range(200, 216))]
SIZES = [0, 1, 2, 15, 16, 17, 31, 32, 33, 47, 48, 63, 64, 65, 68, 127, 128, 129, 255, 256, 1000, 4099]


@pytest.fixture(params=["aesni", "table"])
def impl(request, monkeypatch):
    """The product library's host cipher, and the table cipher through the tuning build."""
    if request.param == "aesni":
        if aes.host_impl() != "aesni":
            pytest.skip("this CPU has no AES-NI")
        yield "aesni"
        return
    monkeypatch.setenv("DN_AES_HOST", "table")
    with _native.library(_native.TUNING_LIB):
        assert aes.host_impl() == "table"
        yield "table"


def rand_bytes(n: int, seed: int) -> bytes:
    return np.random.default_rng(seed).integers(0, 256, n, dtype=np.uint8).tobytes()


def want_text(key, nonce, data) -> bytes:
    return base64.b64encode(nonce + c_oracle.aes_ctr(key, nonce, data))


@pytest.mark.parametrize("key,ct", FIPS197)
def test_fips197_block(impl, key, ct):
    # one CTR block over a zero message at counter = the plaintext block is AES(key, PT)
    assert aes.ctr_host(bytes.fromhex(key), PT, bytes(16)).hex() == ct


@pytest.mark.parametrize("key,ct", SP800)
def test_sp800_38a_ctr(impl, key, ct):
    assert aes.ctr_host(bytes.fromhex(key), bytes.fromhex(SP800_IV), bytes.fromhex(SP800_PT)).hex() == ct


def test_openssl_kat(impl):
    kat = load_json("aes_kat.json")
    assert len(kat["cases"]) >= 250
    for c in kat["cases"]:
        got = aes.ctr_host(bytes.fromhex(c["key"]), bytes.fromhex(c["iv"]), bytes.fromhex(c["pt"]))
        assert got.hex() == c["ct"], c


@pytest.mark.parametrize("n", SIZES)
def test_encrypt_decrypt_against_oracle(impl, n):
    data = rand_bytes(n, n)
    for key in KEYS:
        for nonce in NONCES:
            text = aes.encrypt(key, data, nonce=nonce)
            assert text == want_text(key, nonce, data), (len(key), nonce.hex())
            assert aes.decrypt(key, text) == data
            assert aes.decrypt(key, text.decode()) == data


def test_counter_wraps_mod_2_128(impl):
    """The 128-bit counter carries across the 64-bit halves and wraps at 2^128
    (cryptography's CTR), also inside an 8-block AES-NI batch."""
    data = rand_bytes(16 * 40 + 5, 1)
    for nonce in (bytes(8) + b"\xff" * 7 + b"\xf0", b"\xff" * 15 + b"\xf8", b"\xff" * 16):
        assert aes.ctr_host(KEYS[0], nonce, data) == c_oracle.aes_ctr(KEYS[0], nonce, data)


def test_bytes_like_inputs_and_random_nonce():
    key = KEYS[0]
    data = b"delta-node seed share"
    s = aes.encrypt(key, bytearray(data))
    raw = base64.b64decode(s)
    assert len(raw) == 16 + len(data) and raw[16:] == c_oracle.aes_ctr(key, raw[:16], data)
    assert aes.decrypt(bytearray(key), memoryview(s)) == data
    assert aes.encrypt(key, b"abc") != aes.encrypt(key, b"abc")  # os.urandom nonce, as the reference


def _odd_texts(b64: bytes):
    yield b64[:40] + b"\n" + b64[40:]   # b64decode drops characters outside the alphabet
    yield b64.rstrip(b"=")              # missing padding
    yield b64[:8] + b"=" + b64[9:]      # '=' inside
    yield b64[:-4] + b"QQ=="            # another canonical tail
    yield b64[:-4] + b"QR=="            # nonzero bits under the padding (b64decode ignores them)
    yield b64[:10] + b"*" + b64[11:]
    yield base64.b64encode(b"short nonce")
    yield b""
    yield b"===="


def ref_decrypt(key, text: bytes) -> bytes:
    """aes.py:17-23 with the oracle cipher (the nonce-size check is cryptography's)."""
    raw = base64.b64decode(text)
    if len(raw[:16]) != 16:
        raise ValueError("Invalid nonce size")
    return c_oracle.aes_ctr(key, raw[:16], raw[16:])


def test_noncanonical_text_behaves_like_reference(impl):
    key, nonce = KEYS[0], NONCES[4]
    for n in (0, 5, 68, 100):
        data = rand_bytes(n, n)
        for text in _odd_texts(want_text(key, nonce, data)):
            try:
                want = ref_decrypt(key, text)
            except ValueError as e:  # binascii.Error is a ValueError
                with pytest.raises(type(e)):
                    aes.decrypt(key, text)
                continue
            assert aes.decrypt(key, text) == want, (n, text[:60])
    with pytest.raises(binascii.Error):
        aes.decrypt(key, want_text(key, nonce, b"x" * 40)[:-1])
    with pytest.raises(ValueError, match="ASCII"):
        aes.decrypt(key, "é" * 24)


def test_reference_errors():
    with pytest.raises(ValueError, match=r"Invalid key size \(40\) for AES"):
        aes.encrypt(b"short", b"data")
    with pytest.raises(ValueError, match="Invalid key size"):
        aes.decrypt(bytes(33), b"")
    with pytest.raises(ValueError, match="nonce"):
        aes.encrypt(bytes(32), b"x", nonce=b"abc")
    with pytest.raises(TypeError):
        aes.encrypt("not bytes", b"x")
    with pytest.raises(TypeError):
        aes.encrypt(bytes(32), "a str is not bytes")


@pytest.mark.parametrize("nbytes", [16, 24, 32])
def test_host_key_schedule_equals_the_device_schedule(nbytes):
    L = aes_mod._lib()
    for seed in range(16):
        key = bytes((seed * 59 + 13 * i + 7) & 0xFF for i in range(nbytes))
        a, b = (ctypes.c_uint32 * 60)(), (ctypes.c_uint32 * 60)()
        na, nb = ctypes.c_int32(), ctypes.c_int32()
        assert L.dn_aes_expand_key(key, nbytes, a, ctypes.byref(na)) == 0
        assert L.dn_aes_expand_key_host(key, nbytes, b, ctypes.byref(nb)) == 0
        assert list(a) == list(b) and na.value == nb.value == nbytes // 4 + 6


def test_host_c_abi_argument_errors():
    L = aes_mod._lib()
    key, iv = bytes(range(32)), bytes(16)
    assert L.dn_aes_ctr_host(key, 20, iv, b"x", None, 1) == _native.DN_ERR_ARG
    assert "Invalid key size (160) for AES." in _native.last_error()
    assert L.dn_aes_ctr_host(key, 32, None, b"x", None, 1) == _native.DN_ERR_ARG
    assert L.dn_aes_encrypt_host(key, 32, None, b"x", 1, None, 0) == _native.DN_ERR_ARG
    out, n = ctypes.create_string_buffer(64), ctypes.c_uint64()
    assert L.dn_aes_decrypt_host(key, 32, b"A" * 23, 23, 0, out, 64, ctypes.byref(n)) == _native.DN_ERR_RETRY
    assert L.dn_aes_decrypt_host(key, 32, b"A" * 64, 64, 0, out, 1, ctypes.byref(n)) == _native.DN_ERR_ARG
    hx = want_text(key, iv, b"hello").hex().encode()
    assert L.dn_aes_decrypt_host(key, 32, hx, len(hx), 1, out, 64, ctypes.byref(n)) == _native.DN_OK
    assert out.raw[: n.value] == b"hello"
    assert L.dn_aes_decrypt_host(key, 32, b"zz" + hx[2:], len(hx), 1, out, 64, ctypes.byref(n)) == _native.DN_ERR_RETRY


def test_large_message_without_a_device_stays_on_the_host(monkeypatch):
    """Above HOST_MAX_BYTES the byte API uses the GPU only when one is visible."""
    monkeypatch.setattr(_native, "has_device", lambda: False)
    monkeypatch.setattr(aes_mod, "HOST_MAX_BYTES", 100)
    data = rand_bytes(5000, 7)
    text = aes.encrypt(KEYS[0], data, nonce=NONCES[2])
    assert text == want_text(KEYS[0], NONCES[2], data)
    assert aes.decrypt(KEYS[0], text) == data


@pytest.mark.parametrize("n", [68, 33])
def test_per_call_latency(n):
    """One share per call, as the reference's callers do: <= 10 us each way
    (best of five batches of 2000 calls, the Python wrapper included)."""
    key, data = os.urandom(32), os.urandom(n)
    text = aes.encrypt(key, data)
    enc = dec = float("inf")
    for _ in range(5):
        t0 = time.perf_counter()
        for _ in range(2000):
            aes.encrypt(key, data)
        t1 = time.perf_counter()
        for _ in range(2000):
            aes.decrypt(key, text)
        t2 = time.perf_counter()
        enc, dec = min(enc, (t1 - t0) / 2000), min(dec, (t2 - t1) / 2000)
    assert aes.decrypt(key, text) == data
    assert enc <= 10e-6 and dec <= 10e-6, (enc * 1e6, dec * 1e6)
