"""`delta_node.serialize` subset used by the Shamir path.

Reference: delta_node/serialize/__init__.py re-exports hex.py's codec
(`int_to_bytes`, `bytes_to_int`, `bytes_to_hex`, `hex_to_bytes`); the
pickle/npz helpers there are outside the hot path and not provided.
"""
from .hex import bytes_to_hex, bytes_to_int, hex_to_bytes, int_to_bytes

__all__ = ["int_to_bytes", "bytes_to_int", "bytes_to_hex", "hex_to_bytes"]
