"""calc_commitment (reference: delta_node/utils/commitment.py:1-12).

SHA-256 of a byte string, or of the concatenation of the chunks an IO[bytes]
(or any iterable of byte chunks) yields.  This is the file-commitment helper of
the upload path, not part of the hot path: hashlib on the host, as the
reference does.
"""
from __future__ import annotations

from hashlib import sha256
from typing import IO, Union

__all__ = ["calc_commitment"]


def calc_commitment(content: Union[bytes, IO[bytes]]) -> bytes:
    h = sha256()
    if isinstance(content, bytes):
        h.update(content)
    else:
        for chunk in content:
            h.update(chunk)
    return h.digest()
