"""Share-envelope cipher (second half) on the CPU: the
oracle (oracle/aes_oracle.c) against independent vectors, the product
library's host key schedule against the oracle, and the reference's argument
errors before any device work.

Independent vectors: FIPS-197 Appendix C (AES-128/192/256 block), NIST
SP 800-38A F.5.1 / F.5.5 (CTR-AES128 / CTR-AES256), and `openssl enc
-aes-*-ctr` outputs (tests/golden/aes_kat.json, make_golden_aes.py) — OpenSSL
is the library the reference's `cryptography` wraps (crypto/aes/aes.py:4).
"""
import base64

import pytest
import torch

from delta_node.crypto import aes
from delta_node.crypto.aes import aes as aes_mod
from golden.fixtures import load_json
from oracle import c_oracle

PT = bytes.fromhex("00112233445566778899aabbccddeeff")
FIPS197 = [
    ("000102030405060708090a0b0c0d0e0f", "69c4e0d86a7b0430d8cdb78070b4c55a"),
    ("000102030405060708090a0b0c0d0e0f1011121314151617", "dda97ca4864cdfe06eaf70a0ec0d7191"),
    ("000102030405060708090a0b0c0d0e0f101112131415161718191a1b1c1d1e1f", "8ea2b7ca516745bfeafc49904b496089"),
]
SP800_IV = "f0f1f2f3f4f5f6f7f8f9fafbfcfdfeff"
SP800_PT = ("6bc1bee22e409f96e93d7e117393172a" "ae2d8a571e03ac9c9eb76fac45af8e51"
            "30c81c46a35ce411e5fbc1191a0a52ef" "f69f2445df4f9b17ad2b417be66c3710")
SP800 = [
    ("2b7e151628aed2a6abf7158809cf4f3c",
     "874d6191b620e3261bef6864990db6ce" "9806f66b7970fdff8617187bb9fffdff"
     "5ae4df3edbd5d35e5b4f09020db03eab" "1e031dda2fbe03d1792170a0f3009cee"),
    ("603deb1015ca71be2b73aef0857d77811f352c073b6108d72d9810a30914dff4",
     "601ec313775789a5b7a7f504bbf3d228" "f443e3ca4d62b59aca84e990cacaf5c5"
     "2b0930daa23de94ce87017ba2d84988d" "dfc9c58db67aada613c2dd08457941a6"),
]


def test_sbox_entries():
    assert [c_oracle.aes_sbox(x) for x in (0x00, 0x01, 0x53, 0xFF)] == [0x63, 0x7C, 0xED, 0x16]


@pytest.mark.parametrize("key,ct", FIPS197)
def test_fips197_block(key, ct):
    assert c_oracle.aes_block(bytes.fromhex(key), PT).hex() == ct


@pytest.mark.parametrize("key,ct", SP800)
def test_sp800_38a_ctr(key, ct):
    assert c_oracle.aes_ctr(bytes.fromhex(key), bytes.fromhex(SP800_IV), bytes.fromhex(SP800_PT)).hex() == ct


def test_openssl_kat():
    kat = load_json("aes_kat.json")
    assert len(kat["cases"]) >= 250
    for c in kat["cases"]:
        got = c_oracle.aes_ctr(bytes.fromhex(c["key"]), bytes.fromhex(c["iv"]), bytes.fromhex(c["pt"]))
        assert got.hex() == c["ct"], c


@pytest.mark.parametrize("nbytes", [16, 24, 32])
def test_host_key_schedule_matches_oracle(nbytes):
    for seed in range(4):
        key = bytes((seed * 37 + 11 * i + 5) & 0xFF for i in range(nbytes))
        rk = c_oracle.aes_expand(key)
        assert aes.expand_key(key) == [int.from_bytes(rk[4 * i:4 * i + 4], "big") for i in range(len(rk) // 4)]


def test_text_lengths():
    L = aes_mod._lib()
    for n in (0, 1, 2, 3, 31, 32, 33, 1000):
        b64 = len(base64.b64encode(bytes(16 + n)))
        assert L.dn_aes_encrypt_len(n, 0) == b64 and L.dn_aes_encrypt_len(n, 1) == 2 * b64
        cap = L.dn_aes_decrypt_capacity(b64, 0)
        assert n <= cap < n + 3
        assert L.dn_aes_decrypt_capacity(2 * b64, 1) == cap
    for bad in (0, 4, 20, 23, 25, 26):  # shorter than a nonce, or not a multiple of 4
        assert L.dn_aes_decrypt_capacity(bad, 0) == 0
    assert L.dn_aes_decrypt_capacity(49, 1) == 0  # odd number of hex digits


def test_reference_errors_before_device():
    with pytest.raises(ValueError, match=r"Invalid key size \(40\) for AES"):
        aes.encrypt(b"short", b"data")
    with pytest.raises(ValueError, match="Invalid key size"):
        aes.decrypt(bytes(33), b"")
    with pytest.raises(ValueError, match="nonce"):
        aes.encrypt(bytes(32), b"x", nonce=b"abc")
    with pytest.raises(TypeError):
        aes.encrypt("not bytes", b"x")
    with pytest.raises(ValueError, match="Invalid key size"):
        aes.expand_key(bytes(20))


def test_byte_api_runs_without_a_device():
    """aes.encrypt / aes.decrypt of a share need no GPU (csrc/host_aes.cpp)."""
    key = bytes(range(32))
    text = aes.encrypt(key, b"data", nonce=bytes(16))
    assert text == base64.b64encode(bytes(16) + c_oracle.aes_ctr(key, bytes(16), b"data"))
    assert aes.decrypt(key, text) == b"data"


def test_c_abi_argument_errors_before_any_device_work():
    """The C-ABI's host-side checks (dn_aes.h): they return before touching a
    device pointer, so fake pointers are safe here."""
    from delta_node.crypto.shamir import _native

    L = aes_mod._lib()
    key, iv = bytes(range(32)), bytes(16)
    assert L.dn_aes_encrypt(key, 20, iv, 16, 32, 4096, 0, None) == _native.DN_ERR_ARG
    assert "Invalid key size (160) for AES." in _native.last_error()
    assert L.dn_aes_encrypt(key, 32, iv, 16, 32, 4097, 1, None) == _native.DN_ERR_ARG  # misaligned output
    assert "16-byte aligned" in _native.last_error()
    assert L.dn_aes_encrypt(key, 32, None, 16, 32, 4096, 0, None) == _native.DN_ERR_ARG
    assert L.dn_aes_encrypt(key, 32, iv, None, 32, 4096, 0, None) == _native.DN_ERR_ARG
    assert L.dn_aes_ctr(key, 32, None, 16, 4096, 64, None) == _native.DN_ERR_ARG
    assert L.dn_aes_ctr(key, 32, iv, 16, 4096, 0, None) == _native.DN_OK  # nothing to do
    assert L.dn_aes_decrypt(key, 32, 16, 23, 0, 4096, 64, 8, 8, None) == _native.DN_ERR_RETRY  # < a nonce
    assert L.dn_aes_decrypt(key, 32, 16, 49, 1, 4096, 64, 8, 8, None) == _native.DN_ERR_RETRY  # odd hex
    assert L.dn_aes_decrypt(key, 32, 16, 64, 0, 4096, 1, 8, 8, None) == _native.DN_ERR_ARG  # capacity 1 < 32
    assert L.dn_aes_decrypt(key, 16, 16, 64, 0, None, 64, 8, 8, None) == _native.DN_ERR_ARG  # null output
