"""The share envelope on the GPU (second half).

Reference (delta-mpc/delta-node), delta_node/crypto/aes/aes.py:8-23::

    encrypt(key, data) = b64encode(nonce + Cipher(AES(key), CTR(nonce)).encryptor().update(data)),
                         nonce = os.urandom(16)
    decrypt(key, data) = Cipher(AES(key), CTR(raw[:16])).decryptor().update(raw[16:]),
                         raw = b64decode(data)

(`cryptography` -> OpenSSL; the runner's keys are 32-byte ECDH digests,
crypto/ecdhe/ecdhe.py:23-34), plus the hex layer the runner and coordinator
put around it in the JSON of upload_secret_shares (serialize.bytes_to_hex /
hex_to_bytes, serialize/hex.py:11-41; runner/horizontal/commu.py:23-49;
app/v1/coord.py:93-94).

`encrypt` / `decrypt` keep the reference's signatures (bytes in, bytes out).
`encrypt_vec` / `decrypt_vec` take and return uint8 device tensors — for a
vector share, the packed `_share_to_bytes` records of `crypto.shamir.codec` —
and with ``hex=True`` include the hex layer: ``encrypt_vec(k, r, hex=True)`` is
the ASCII of ``serialize.bytes_to_hex(encrypt(k, r))``.  AES, base64 and hex
run in one kernel (dn_aes_encrypt / dn_aes_decrypt, csrc/aes_envelope.hip).

Text that is not canonical base64 / hex (whitespace, missing padding, stray
'=' or characters outside the alphabet) is parsed on the host with the
reference's own calls (bytes.fromhex, base64.b64decode), so the result — or
the exception — is the reference's; the keystream still comes from the GPU
(dn_aes_ctr).  There is no CPU cipher.
"""
from __future__ import annotations

import base64
import ctypes
import os
from typing import List, Optional, Union

from ..shamir import _native

EXPORTS = ("dn_aes_expand_key", "dn_aes_ctr", "dn_aes_encrypt_len", "dn_aes_encrypt", "dn_aes_decrypt_capacity",
           "dn_aes_decrypt")
def _lib() -> ctypes.CDLL:
    L = _native.lib()
    if not getattr(L, "_dn_aes_bound", False):  # argtypes, once per loaded library
        vp, u64, i32, cp = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int, ctypes.c_char_p
        L.dn_aes_expand_key.restype = i32
        L.dn_aes_expand_key.argtypes = [cp, i32, ctypes.POINTER(ctypes.c_uint32), ctypes.POINTER(ctypes.c_int32)]
        L.dn_aes_ctr.restype = i32
        L.dn_aes_ctr.argtypes = [cp, i32, cp, vp, vp, u64, vp]
        L.dn_aes_encrypt_len.restype = u64
        L.dn_aes_encrypt_len.argtypes = [u64, i32]
        L.dn_aes_encrypt.restype = i32
        L.dn_aes_encrypt.argtypes = [cp, i32, cp, vp, u64, vp, i32, vp]
        L.dn_aes_decrypt_capacity.restype = u64
        L.dn_aes_decrypt_capacity.argtypes = [u64, i32]
        L.dn_aes_decrypt.restype = i32
        L.dn_aes_decrypt.argtypes = [cp, i32, vp, u64, i32, vp, u64, vp, vp, vp]
        L._dn_aes_bound = True
    return L


def _key(key) -> bytes:
    """cryptography's checks of algorithms.AES: bytes-like, 128 / 192 / 256 bits."""
    if not isinstance(key, (bytes, bytearray, memoryview)):
        raise TypeError("key must be bytes-like")
    key = bytes(key)
    if len(key) * 8 not in (128, 192, 256):
        raise ValueError(f"Invalid key size ({len(key) * 8}) for AES.")
    return key


def _nonce(nonce) -> bytes:
    nonce = os.urandom(16) if nonce is None else bytes(nonce)
    if len(nonce) != 16:
        raise ValueError(f"Invalid nonce size ({len(nonce)}) for CTR.")
    return nonce


def expand_key(key) -> List[int]:
    """Round keys from the library's host key schedule (FIPS-197 w[i], big-endian words)."""
    k = _key(key)
    rk = (ctypes.c_uint32 * 60)()
    nr = ctypes.c_int32()
    _native.check(_lib().dn_aes_expand_key(k, len(k), rk, ctypes.byref(nr)))
    return list(rk[: 4 * (nr.value + 1)])


def _u8(t, what: str):
    import torch

    if not (isinstance(t, torch.Tensor) and t.dtype == torch.uint8 and t.is_cuda and t.dim() == 1
            and t.is_contiguous()):
        raise ValueError(f"{what}: expected a contiguous 1-D uint8 device tensor")
    return t


def _ptr(t) -> Optional[int]:
    return t.data_ptr() if t.numel() else None


def ctr_vec(key, nonce: bytes, data, out=None):
    """`Cipher(AES(key), CTR(nonce)).encryptor().update(data)` (either direction) of a device byte vector."""
    import torch

    k, iv = _key(key), _nonce(nonce)
    _u8(data, "ctr_vec")
    if out is None:
        out = torch.empty_like(data)
    _native.check(_lib().dn_aes_ctr(k, len(k), iv, _ptr(data), _ptr(out), data.numel(), _native.stream_ptr()))
    return out


def encrypt_vec(key, data, *, nonce: Optional[bytes] = None, hex: bool = False):
    """`aes.encrypt(key, data)` of a device byte vector -> uint8 device tensor of
    the base64 text, or with hex=True of "0x" + its hex (serialize.bytes_to_hex)."""
    import torch

    k, iv = _key(key), _nonce(nonce)
    _u8(data, "encrypt_vec")
    L = _lib()
    n = data.numel()
    size = int(L.dn_aes_encrypt_len(n, int(hex)))
    lead = 16 if hex else 0  # the kernel writes from a 16-byte boundary; "0x" goes just in front
    buf = torch.empty(lead + size, dtype=torch.uint8, device=data.device)
    _native.check(L.dn_aes_encrypt(k, len(k), iv, _ptr(data), n, buf.data_ptr() + lead, int(hex),
                                   _native.stream_ptr()))
    if not hex:
        return buf
    buf[lead - 2] = ord("0")
    buf[lead - 1] = ord("x")
    return buf[lead - 2:]


def decrypt_vec(key, text, *, hex: bool = False):
    """`aes.decrypt(key, text)` of a device text (base64; hex=True: hex_to_bytes of
    it first, with or without "0x") -> uint8 device tensor of the plaintext."""
    import torch

    k = _key(key)
    _u8(text, "decrypt_vec")
    ptr, n_text = text.data_ptr(), text.numel()
    if hex and n_text >= 2 and bytes(text[:2].cpu().numpy()) == b"0x":
        ptr, n_text = ptr + 2, n_text - 2
    L = _lib()
    cap = int(L.dn_aes_decrypt_capacity(n_text, int(hex)))
    if cap:
        out = torch.empty(cap, dtype=torch.uint8, device=text.device)
        meta = torch.zeros(2, dtype=torch.int64, device=text.device)  # [plaintext bytes, non-canonical flag]
        rc = L.dn_aes_decrypt(k, len(k), ptr, n_text, int(hex), out.data_ptr(), cap, meta.data_ptr(),
                              meta.data_ptr() + 8, _native.stream_ptr())
        if rc != _native.DN_ERR_RETRY:
            _native.check(rc)
            out_len, bad = meta.tolist()
            if not bad:
                return out[:out_len]
    return _decrypt_parsed_on_host(k, text, hex)


def _decrypt_parsed_on_host(k: bytes, text, hex: bool):
    """Non-canonical text: parsed by the reference's own calls (hex.py:29-41,
    aes.py:18-19), so errors are the reference's; the keystream is the GPU's."""
    import torch

    from ... import serialize

    raw_text = bytes(text.cpu().numpy())
    if hex:
        raw_text = serialize.hex_to_bytes(raw_text.decode("ascii"))
    raw = base64.b64decode(raw_text)
    iv = _nonce(raw[:16])
    ct = raw[16:]
    if not ct:
        return torch.empty(0, dtype=torch.uint8, device=text.device)
    return ctr_vec(k, iv, torch.frombuffer(bytearray(ct), dtype=torch.uint8).to(text.device))


def _to_device(data: bytes):
    import torch

    dev = _native.require_device()
    if not data:
        return torch.empty(0, dtype=torch.uint8, device=dev)
    return torch.frombuffer(bytearray(data), dtype=torch.uint8).to(dev)


def encrypt(key: bytes, data: bytes, *, nonce: Optional[bytes] = None) -> bytes:
    """aes.py:8-14: b64encode(nonce + AES-CTR(key, nonce)(data)); nonce = os.urandom(16) by default."""
    _key(key)
    if nonce is not None:
        _nonce(nonce)
    return bytes(encrypt_vec(key, _to_device(bytes(data)), nonce=nonce).cpu().numpy())


def decrypt(key: bytes, data: Union[bytes, str]) -> bytes:
    """aes.py:17-23."""
    _key(key)
    if isinstance(data, str):
        data = data.encode("ascii")
    return bytes(decrypt_vec(key, _to_device(bytes(data))).cpu().numpy())
