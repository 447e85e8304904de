"""Golden-fixture helpers shared by `make_golden.py` (generation) and the tests.

Test infrastructure only.  Defines:

* the canonical limb form of a field element (17 little-endian u32 limbs, the
  top limb holding bits 512..520), and
* the layout-independent "checksum of checksums" used to pin full-size outputs:
  vectors are cut into chunks of ``DIGEST_CHUNK`` elements; for each chunk the
  bytes of every vector's 16 u32 limb planes followed by its u16 top-limb plane
  (little endian, plane-major inside the chunk) are hashed with SHA-256, and
  the final digest is SHA-256 over the concatenated chunk digests.
"""
from __future__ import annotations

import hashlib
import json
import os
from concurrent.futures import ThreadPoolExecutor
from typing import Iterable, List, Sequence

import numpy as np

P = (1 << 521) - 1
DIGEST_CHUNK = 1 << 16
HERE = os.path.dirname(os.path.abspath(__file__))
INT64_MIN = -(1 << 63)
INT64_MAX = (1 << 63) - 1


def secrets_int64(seed: int, n: int) -> np.ndarray:
    """Synthetic int64 secrets: full int64 range, numpy PCG64 seeded."""
    rng = np.random.default_rng(seed)
    return rng.integers(INT64_MIN, INT64_MAX, size=n, endpoint=True, dtype=np.int64)


def ints_to_limbs(vals: Sequence[int]) -> np.ndarray:
    """Python ints in [0, 2^521) -> uint32 [len, 17] limbs (little endian)."""
    buf = b"".join(int(v).to_bytes(68, "little") for v in vals)
    return np.frombuffer(buf, dtype="<u4").reshape(len(vals), 17).copy()


def limbs_to_ints(limbs: np.ndarray) -> List[int]:
    limbs = np.ascontiguousarray(limbs, dtype="<u4").reshape(-1, 17)
    raw = limbs.tobytes()
    return [int.from_bytes(raw[i * 68:(i + 1) * 68], "little") for i in range(limbs.shape[0])]


def _chunk_bytes(planes: np.ndarray, lo: int, hi: int) -> bytes:
    """planes: uint32 [S, 17, N] -> canonical bytes of elements [lo, hi)."""
    parts = []
    for s in range(planes.shape[0]):
        parts.append(np.ascontiguousarray(planes[s, :16, lo:hi], dtype="<u4").tobytes())
        parts.append(np.ascontiguousarray(planes[s, 16, lo:hi]).astype("<u2").tobytes())
    return b"".join(parts)


def chunk_digests(planes: np.ndarray, threads: int = 8) -> List[bytes]:
    """uint32 [S, 17, N] limb planes -> list of per-chunk SHA-256 digests."""
    n = planes.shape[2]
    starts = list(range(0, n, DIGEST_CHUNK))

    def one(lo):
        return hashlib.sha256(_chunk_bytes(planes, lo, min(n, lo + DIGEST_CHUNK))).digest()

    if threads <= 1 or len(starts) == 1:
        return [one(lo) for lo in starts]
    with ThreadPoolExecutor(threads) as ex:
        return list(ex.map(one, starts))


def combine_digests(chunks: Iterable[bytes]) -> str:
    return hashlib.sha256(b"".join(chunks)).hexdigest()


def planes_digest(planes: np.ndarray) -> str:
    return combine_digests(chunk_digests(planes))


def manifest() -> dict:
    with open(os.path.join(HERE, "manifest.json")) as f:
        return json.load(f)


def load_npz(name: str):
    return np.load(os.path.join(HERE, name), allow_pickle=False)


def load_json(name: str):
    with open(os.path.join(HERE, name)) as f:
        return json.load(f)


def unpack_share_bytes(flat: np.ndarray, offsets: np.ndarray, i: int) -> bytes:
    return flat[offsets[i]:offsets[i + 1]].tobytes()
