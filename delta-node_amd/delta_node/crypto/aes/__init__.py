"""`delta_node.crypto.aes` (reference: delta_node/crypto/aes/__init__.py:1) — the share envelope on the GPU."""
from .aes import EXPORTS, ctr_vec, decrypt, decrypt_vec, encrypt, encrypt_vec, expand_key

__all__ = ["encrypt", "decrypt", "encrypt_vec", "decrypt_vec", "ctr_vec", "expand_key", "EXPORTS"]
