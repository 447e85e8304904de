"""Pure-Python restatement of the reference mask PRG — TEST INFRASTRUCTURE ONLY.

Reference: delta_node/utils/arr.py:20-28

    rng = np.random.default_rng(seed if int else list(seed_bytes))
    mask = rng.integers(0, 2**47 - 1, size=shape, dtype=np.int64)

i.e. numpy's SeedSequence (bit_generator.pyx: hashmix/mix/mix_entropy/
generate_state) -> PCG64 (pcg64.h: 128-bit LCG, XSL-RR output; seeded by
pcg64_set_seed -> pcg_setseq_128_srandom_r) -> Generator.integers int64 path
(_bounded_integers: random_bounded_uint64_fill -> bounded_lemire_uint64).
numpy is a pinned dependency of the reference (requirements.txt) and is
present here; this restatement is checked against it bit for bit
(tests/test_mask_oracle.py) and used where the stream must be inspected
(raw draws, rejections), while numpy itself is the checker at full size.
Also restates delta_node/utils/precision.py:5-15 (fix/unfix_precision).
"""
from __future__ import annotations

from typing import List, Sequence, Tuple, Union

import numpy as np

M32 = 0xFFFFFFFF
M64 = (1 << 64) - 1
M128 = (1 << 128) - 1
INIT_A, MULT_A = 0x43B0D7E5, 0x931E8875
INIT_B, MULT_B = 0x8B51F9DD, 0x58F38DED
MIX_MULT_L, MIX_MULT_R = 0xCA01F9DD, 0x4973F715
XSHIFT = 16
POOL = 4
PCG_MULT = (0x2360ED051FC65DA4 << 64) | 0x4385DF649FCCF645


def entropy_words(seed: Union[int, bytes, Sequence[int]]) -> List[int]:
    """SeedSequence entropy -> uint32 words (_coerce_to_uint32_array)."""
    def int_words(v: int) -> List[int]:
        if v < 0:
            raise ValueError("expected non-negative integer")
        if v == 0:
            return [0]
        out = []
        while v:
            out.append(v & M32)
            v >>= 32
        return out

    if isinstance(seed, int):
        return int_words(seed)
    words: List[int] = []
    for v in (list(seed) if isinstance(seed, (bytes, bytearray)) else seed):
        words.extend(int_words(int(v)))
    return words


def _hashmix(value: int, hc: List[int]) -> int:
    value = (value ^ hc[0]) & M32
    hc[0] = (hc[0] * MULT_A) & M32
    value = (value * hc[0]) & M32
    return value ^ (value >> XSHIFT)


def _mix(x: int, y: int) -> int:
    r = (MIX_MULT_L * x - MIX_MULT_R * y) & M32
    return r ^ (r >> XSHIFT)


def seed_pool(words: Sequence[int]) -> List[int]:
    hc = [INIT_A]
    pool = [_hashmix(words[i] if i < len(words) else 0, hc) for i in range(POOL)]
    for s in range(POOL):
        for d in range(POOL):
            if s != d:
                pool[d] = _mix(pool[d], _hashmix(pool[s], hc))
    for s in range(POOL, len(words)):
        for d in range(POOL):
            pool[d] = _mix(pool[d], _hashmix(words[s], hc))
    return pool


def generate_state_u64(pool: Sequence[int], n64: int) -> List[int]:
    hc = INIT_B
    w32 = []
    for i in range(2 * n64):
        v = pool[i % POOL] ^ hc
        hc = (hc * MULT_B) & M32
        v = (v * hc) & M32
        w32.append(v ^ (v >> XSHIFT))
    return [w32[2 * i] | (w32[2 * i + 1] << 32) for i in range(n64)]


def pcg64_init(seed) -> Tuple[int, int]:
    """(state, inc) numpy's PCG64 holds right after seeding (before any draw)."""
    v = generate_state_u64(seed_pool(entropy_words(seed)), 4)
    s = (v[0] << 64) | v[1]
    i = (v[2] << 64) | v[3]
    inc = ((i << 1) | 1) & M128
    state = (0 * PCG_MULT + inc) & M128
    state = (state + s) & M128
    state = (state * PCG_MULT + inc) & M128
    return state, inc


def pcg64_next(state: int, inc: int) -> Tuple[int, int]:
    state = (state * PCG_MULT + inc) & M128
    hi, lo = state >> 64, state & M64
    x, rot = hi ^ lo, hi >> 58
    return state, ((x >> rot) | (x << ((64 - rot) & 63))) & M64


def bounded_int64(seed, n: int, low: int, high: int, return_raw: bool = False):
    """Generator.integers(low, high, n, int64) for high - low - 1 > 2^32 - 1."""
    rng = high - 1 - low
    assert rng > M32, "only the 64-bit Lemire path is restated"
    excl = rng + 1
    threshold = (M64 - rng) % excl
    state, inc = pcg64_init(seed)
    out, raw, rejects = [], 0, []
    while len(out) < n:
        state, x = pcg64_next(state, inc)
        m = x * excl
        if (m & M64) < threshold:
            rejects.append(raw)
        else:
            out.append(low + (m >> 64))
        raw += 1
    return (out, rejects) if return_raw else out


def make_mask(seed: Union[int, bytes], shape) -> np.ndarray:
    n = int(np.prod(shape)) if not isinstance(shape, int) else shape
    return np.array(bounded_int64(seed, n, 0, 2 ** 47 - 1), dtype=np.int64).reshape(shape)


def make_mask_numpy(seed: Union[int, bytes], shape) -> np.ndarray:
    """The reference call itself (utils/arr.py:20-28), numpy being the dependency."""
    rng = np.random.default_rng(seed if isinstance(seed, int) else list(seed))
    return rng.integers(0, 2 ** 47 - 1, size=shape, dtype=np.int64)


def fix_precision(arr: np.ndarray, precision: int) -> np.ndarray:
    """precision.py:5-9: float64 * 10^p, truncated to int64 (C cast)."""
    return (np.asarray(arr).astype(np.float64) * (10 ** precision)).astype(np.int64)


def unfix_precision(arr: np.ndarray, precision: int) -> np.ndarray:
    """precision.py:12-15."""
    return np.asarray(arr).astype(np.float64) / (10 ** precision)
