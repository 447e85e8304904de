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
(dn_aes_ctr).

The byte API (`encrypt` / `decrypt`, one share per call in the reference's
callers: runner/horizontal/agg.py:192-196, :258, :265) runs on the calling
core — dn_aes_encrypt_host / dn_aes_decrypt_host (csrc/host_aes.cpp, AES-NI)
— for messages up to `HOST_MAX_BYTES` and whenever no HIP device is visible: a
~70-byte share costs ~1 us there against ~100 us of launch and copies.  Larger
byte messages on a GPU node, and every `*_vec` call, run on the device.
"""
from __future__ import annotations

import base64
import ctypes
import os
from typing import List, Optional, Union

from ..shamir import _native

EXPORTS = ("dn_aes_expand_key", "dn_aes_ctr", "dn_aes_encrypt_len", "dn_aes_encrypt", "dn_aes_decrypt_capacity",
           "dn_aes_decrypt", "dn_aes_ctr_host", "dn_aes_encrypt_host", "dn_aes_decrypt_host", "dn_aes_host_impl", "dn_aes_expand_key_host")

# byte-API messages up to this size are sealed / opened on the calling core
# even on a GPU node (host AES-NI at ~2-4 GB/s beats H2D + launch + D2H below
# ~1 MiB; the vector API is the device path)
HOST_MAX_BYTES = 1 << 20


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
        L.dn_aes_ctr_host.restype = i32
        L.dn_aes_ctr_host.argtypes = [cp, i32, cp, cp, vp, u64]
        L.dn_aes_encrypt_host.restype = i32
        L.dn_aes_encrypt_host.argtypes = [cp, i32, cp, cp, u64, vp, i32]
        L.dn_aes_decrypt_host.restype = i32
        L.dn_aes_decrypt_host.argtypes = [cp, i32, cp, u64, i32, vp, u64, ctypes.POINTER(ctypes.c_uint64)]
        L.dn_aes_expand_key_host.restype = i32
        L.dn_aes_expand_key_host.argtypes = [cp, i32, ctypes.POINTER(ctypes.c_uint32), ctypes.POINTER(ctypes.c_int32)]
        L.dn_aes_host_impl.restype = i32
        L.dn_aes_host_impl.argtypes = []
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


_PREFIX = {}  # device index -> the two bytes "0x" on that device


def encrypt_buffer(n: int, hex: bool = False, device=None):
    """A buffer `encrypt_vec(..., out=buf)` can fill for an n-byte message
    (reused across calls of that size: no allocation per call)."""
    import torch

    lead = 16 if hex else 0
    dev = device if device is not None else _native.require_device()
    return torch.empty(lead + int(_lib().dn_aes_encrypt_len(n, int(hex))), dtype=torch.uint8, device=dev)


def encrypt_vec(key, data, *, nonce: Optional[bytes] = None, hex: bool = False, out=None):
    """`aes.encrypt(key, data)` of a device byte vector -> uint8 device tensor of
    the base64 text, or with hex=True of "0x" + its hex (serialize.bytes_to_hex).
    out: a buffer from encrypt_buffer(data.numel(), hex) (the result is a view of it)."""
    import torch

    k, iv = _key(key), _nonce(nonce)
    _u8(data, "encrypt_vec")
    L = _lib()
    n = data.numel()
    size = int(L.dn_aes_encrypt_len(n, int(hex)))
    lead = 16 if hex else 0  # the kernel writes from a 16-byte boundary; "0x" goes just in front
    if out is None:
        buf = torch.empty(lead + size, dtype=torch.uint8, device=data.device)
    else:
        buf = _u8(out, "encrypt_vec out")
        if buf.numel() < lead + size or buf.device != data.device or (buf.data_ptr() + lead) % 16:
            raise ValueError("encrypt_vec: out must come from encrypt_buffer(n, hex) on the data's device")
    _native.check(L.dn_aes_encrypt(k, len(k), iv, _ptr(data), n, buf.data_ptr() + lead, int(hex),
                                   _native.stream_ptr()))
    if not hex:
        return buf[:size]
    pre = _PREFIX.get(buf.device.index)
    if pre is None:
        pre = _PREFIX[buf.device.index] = torch.tensor([ord("0"), ord("x")], dtype=torch.uint8, device=buf.device)
    buf[lead - 2:lead].copy_(pre)  # one device copy
    return buf[lead - 2:lead + size]


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


def _bytes(data) -> bytes:
    """cryptography's update() takes bytes-like data only (a str raises TypeError)."""
    if isinstance(data, bytes):
        return data
    if isinstance(data, (bytearray, memoryview)):
        return bytes(data)
    raise TypeError("data must be bytes-like")


def ctr_host(key, nonce: bytes, data) -> bytes:
    """`Cipher(AES(key), CTR(nonce)).encryptor().update(data)` on the calling core."""
    k, iv, d = _key(key), _nonce(nonce), _bytes(data)
    out = ctypes.create_string_buffer(len(d))
    _native.check(_lib().dn_aes_ctr_host(k, len(k), iv, d, out, len(d)))
    return out.raw


def _encrypt_host(k: bytes, iv: bytes, d: bytes) -> bytes:
    L = _lib()
    out = ctypes.create_string_buffer(4 * ((len(d) + 18) // 3))
    _native.check(L.dn_aes_encrypt_host(k, len(k), iv, d, len(d), out, 0))
    return out.raw


def _decrypt_host(k: bytes, text: bytes) -> bytes:
    L = _lib()
    cap = int(L.dn_aes_decrypt_capacity(len(text), 0))
    if cap:
        out = ctypes.create_string_buffer(cap)
        n = ctypes.c_uint64()
        rc = L.dn_aes_decrypt_host(k, len(k), text, len(text), 0, out, cap, ctypes.byref(n))
        if rc == _native.DN_OK:
            return out.raw[: n.value]
        if rc != _native.DN_ERR_RETRY:
            _native.check(rc)
    # not canonical base64: the reference's own parse (aes.py:18-19), its errors
    raw = base64.b64decode(text)
    return ctr_host(k, raw[:16], raw[16:])


def host_impl() -> str:
    """"aesni" or "table": the host cipher the byte API uses on this CPU."""
    return "aesni" if _lib().dn_aes_host_impl() else "table"


def encrypt(key: bytes, data: bytes, *, nonce: Optional[bytes] = None) -> bytes:
    """aes.py:8-14: b64encode(nonce + AES-CTR(key, nonce)(data)); nonce = os.urandom(16) by default.
    On the calling core up to HOST_MAX_BYTES (or without a HIP device), else on the GPU."""
    k, iv, d = _key(key), _nonce(nonce), _bytes(data)
    if len(d) <= HOST_MAX_BYTES or not _native.has_device():
        return _encrypt_host(k, iv, d)
    return bytes(encrypt_vec(k, _to_device(d), nonce=iv).cpu().numpy())


def decrypt(key: bytes, data: Union[bytes, str]) -> bytes:
    """aes.py:17-23.  On the calling core up to HOST_MAX_BYTES of text (or
    without a HIP device), else on the GPU."""
    k = _key(key)
    if isinstance(data, str):
        try:
            data = data.encode("ascii")
        except UnicodeEncodeError:
            raise ValueError("string argument should contain only ASCII characters") from None
    text = _bytes(data)
    if len(text) <= HOST_MAX_BYTES or not _native.has_device():
        return _decrypt_host(k, text)
    return bytes(decrypt_vec(k, _to_device(text)).cpu().numpy())
