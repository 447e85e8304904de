"""Integer/byte/hex codec (reference: delta_node/serialize/hex.py:11-50).

`int_to_bytes` is minimal big-endian (0 -> b""), so a share or secret with
leading zero bytes comes back shorter; the Shamir byte API inherits that.
"""
from typing import Optional

__all__ = ["int_to_bytes", "bytes_to_int", "bytes_to_hex", "hex_to_bytes"]


def int_to_bytes(x: int) -> bytes:
    """Minimal big-endian bytes of a non-negative int (hex.py:44-46)."""
    return x.to_bytes(-(-x.bit_length() // 8), "big")


def bytes_to_int(bs: bytes) -> int:
    """Big-endian bytes -> int (hex.py:49-50)."""
    return int.from_bytes(bs, "big")


def bytes_to_hex(src: bytes, with0x: bool = True, length: Optional[int] = None) -> str:
    """Hex string of `src`, optionally left-padded to `length` bytes (hex.py:11-26)."""
    if length is not None:
        assert len(src) <= length, f"input bytes length is too long ({len(src)} > {length})"
    text = src.hex() if length is None else src.hex().rjust(2 * length, "0")
    return ("0x" + text) if with0x else text


def hex_to_bytes(src: str, length: Optional[int] = None) -> bytes:
    """Bytes of a hex string with optional '0x' prefix and padding (hex.py:29-41)."""
    body = src[2:] if src.startswith("0x") else src
    if length is not None:
        assert len(body) <= length * 2, f"input hex string length is too long ({len(body)} > {length * 2})"
        body = body.rjust(2 * length, "0")
    return bytes.fromhex(body)
