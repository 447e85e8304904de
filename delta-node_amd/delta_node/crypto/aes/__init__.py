"""`delta_node.crypto.aes` (reference: delta_node/crypto/aes/__init__.py:1) — the share envelope:
the byte API on the calling core, the vector API on the GPU."""
from .aes import (EXPORTS, HOST_MAX_BYTES, ctr_host, ctr_vec, decrypt, decrypt_vec, encrypt, encrypt_buffer, encrypt_vec,
                  expand_key, host_impl)

__all__ = ["encrypt", "decrypt", "encrypt_vec", "encrypt_buffer", "decrypt_vec", "ctr_vec", "ctr_host", "expand_key", "host_impl",
           "HOST_MAX_BYTES", "EXPORTS"]
