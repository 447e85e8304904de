"""Host-side view of the M521 tiled field-element vector layout.

Layout (include/dn_shamir.h): tiles of 256 elements, 16896 bytes each:
``uint32 lo[16][256]`` (limb i of element w at ``lo[i][w]``) then
``uint16 hi[256]`` (bits 512..520).  66 bytes per element, the minimum for a
521-bit value, so HBM bytes moved equal algorithmic bytes.

These numpy helpers convert between Python ints / limb arrays and that
layout.  They are host-side plumbing for the byte API and for tests; the
per-element arithmetic runs in the HIP kernels.
"""
from __future__ import annotations

from typing import List, Sequence

import numpy as np

PRIME = (1 << 521) - 1
TILE = 256
TILE_BYTES = 66 * TILE
LIMBS = 17


def vec_bytes(n: int) -> int:
    """Bytes of one tiled vector of n elements (== dn_m521_vec_bytes)."""
    return ((n + TILE - 1) // TILE) * TILE_BYTES


def ints_to_limbs(vals: Sequence[int]) -> np.ndarray:
    """Python ints in [0, 2^521) -> uint32 [n, 17] little-endian limbs."""
    buf = b"".join(int(v).to_bytes(68, "little") for v in vals)
    return np.frombuffer(buf, dtype="<u4").reshape(len(vals), LIMBS).copy()


def limbs_to_ints(limbs: np.ndarray) -> List[int]:
    raw = np.ascontiguousarray(limbs, dtype="<u4").reshape(-1, LIMBS).tobytes()
    return [int.from_bytes(raw[i * 68:(i + 1) * 68], "little") for i in range(len(raw) // 68)]


def limbs_to_vec(limbs: np.ndarray) -> np.ndarray:
    """uint32 [n, 17] -> uint8 tiled vector of vec_bytes(n) bytes."""
    limbs = np.asarray(limbs, dtype=np.uint32).reshape(-1, LIMBS)
    n = limbs.shape[0]
    ntiles = (n + TILE - 1) // TILE
    pad = np.zeros((ntiles * TILE, LIMBS), dtype=np.uint32)
    pad[:n] = limbs
    t = pad.reshape(ntiles, TILE, LIMBS)
    out = np.empty((ntiles, TILE_BYTES), dtype=np.uint8)
    out[:, :64 * TILE] = np.ascontiguousarray(t[:, :, :16].transpose(0, 2, 1)).astype("<u4").view(np.uint8).reshape(ntiles, -1)
    out[:, 64 * TILE:] = np.ascontiguousarray(t[:, :, 16]).astype("<u2").view(np.uint8).reshape(ntiles, -1)
    return out.reshape(-1)


def vec_to_limbs(vec: np.ndarray, n: int) -> np.ndarray:
    """uint8 tiled vector -> uint32 [n, 17]."""
    ntiles = (n + TILE - 1) // TILE
    v = np.asarray(vec, dtype=np.uint8).reshape(-1)[: ntiles * TILE_BYTES].reshape(ntiles, TILE_BYTES)
    lo = np.ascontiguousarray(v[:, :64 * TILE]).view("<u4").reshape(ntiles, 16, TILE)
    hi = np.ascontiguousarray(v[:, 64 * TILE:]).view("<u2").reshape(ntiles, TILE)
    out = np.empty((ntiles, TILE, LIMBS), dtype=np.uint32)
    out[:, :, :16] = lo.transpose(0, 2, 1)
    out[:, :, 16] = hi
    return out.reshape(-1, LIMBS)[:n]


def vec_to_planes(vec: np.ndarray, n: int) -> np.ndarray:
    """uint8 tiled vector -> uint32 [17, n] limb planes (for digests)."""
    ntiles = (n + TILE - 1) // TILE
    v = np.asarray(vec, dtype=np.uint8).reshape(-1)[: ntiles * TILE_BYTES].reshape(ntiles, TILE_BYTES)
    lo = np.ascontiguousarray(v[:, :64 * TILE]).view("<u4").reshape(ntiles, 16, TILE)
    hi = np.ascontiguousarray(v[:, 64 * TILE:]).view("<u2").reshape(ntiles, TILE)
    out = np.empty((LIMBS, ntiles * TILE), dtype=np.uint32)
    out[:16] = lo.transpose(1, 0, 2).reshape(16, -1)
    out[16] = hi.reshape(-1)
    return out[:, :n]


def ints_to_vec(vals: Sequence[int]) -> np.ndarray:
    return limbs_to_vec(ints_to_limbs(vals))


def vec_to_ints(vec: np.ndarray, n: int) -> List[int]:
    return limbs_to_ints(vec_to_limbs(vec, n))
