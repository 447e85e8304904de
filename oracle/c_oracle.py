"""ctypes wrapper of liboracle_m521.so (the C restatement).  Test infrastructure only."""
import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(_HERE, "liboracle_m521.so")
_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            raise RuntimeError(f"{LIB} missing: run `make -C oracle` (or __graft_entry__.build())")
        L = ctypes.CDLL(LIB)
        vp, u64, i32 = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int
        L.oracle_draw_coeffs.argtypes = [u64, u64, i32, vp]
        L.oracle_mt_words.argtypes = [u64, u64, vp]
        L.oracle_split.argtypes = [vp, vp, u64, i32, i32, vp]
        L.oracle_reconstruct.argtypes = [vp, vp, i32, u64, vp]
        L.oracle_chacha_block.argtypes = [vp, u64, u64, i32, vp]
        L.oracle_prng_coeffs.argtypes = [vp, u64, i32, u64, u64, i32, vp]
        cp = ctypes.c_char_p
        L.oracle_aes_sbox.argtypes = [ctypes.c_uint8]
        L.oracle_aes_sbox.restype = ctypes.c_uint8
        L.oracle_aes_expand.argtypes = [cp, i32, vp]
        L.oracle_aes_expand.restype = i32
        L.oracle_aes_block.argtypes = [cp, i32, cp, vp]
        L.oracle_aes_ctr.argtypes = [cp, i32, cp, cp, vp, u64]
        for f in (L.oracle_draw_coeffs, L.oracle_mt_words, L.oracle_split, L.oracle_reconstruct,
                  L.oracle_chacha_block, L.oracle_prng_coeffs, L.oracle_aes_block, L.oracle_aes_ctr):
            f.restype = None
        _lib = L
    return _lib


def aes_sbox(x: int) -> int:
    return int(lib().oracle_aes_sbox(x))


def aes_expand(key: bytes) -> bytes:
    """FIPS-197 round keys, 16 (rounds + 1) bytes."""
    buf = ctypes.create_string_buffer(240)
    nr = lib().oracle_aes_expand(key, len(key), buf)
    return buf.raw[: 16 * (nr + 1)]


def aes_block(key: bytes, block: bytes) -> bytes:
    out = ctypes.create_string_buffer(16)
    lib().oracle_aes_block(key, len(key), block, out)
    return out.raw


def aes_ctr(key: bytes, iv: bytes, data: bytes) -> bytes:
    """data XOR the AES-CTR keystream of (key, iv): 128-bit big-endian counter."""
    out = ctypes.create_string_buffer(max(1, len(data)))
    lib().oracle_aes_ctr(key, len(key), iv, bytes(data), out, len(data))
    return out.raw[: len(data)]


def draw_coeffs(seed: int, n: int, tm1: int) -> np.ndarray:
    """Coefficients random.Random(seed) yields for n make_shares calls: uint32 [n, tm1, 17]."""
    out = np.zeros((n, tm1, 17), dtype=np.uint32)
    if n and tm1:
        lib().oracle_draw_coeffs(seed, n, tm1, out.ctypes.data)
    return out


def _key_words(key: bytes) -> np.ndarray:
    assert len(key) == 32
    return np.frombuffer(key, dtype="<u4").copy()


def chacha_block(key: bytes, counter: int, nonce: int, rounds: int = 20) -> np.ndarray:
    """One 16-word keystream block (64-bit counter in words 12-13, nonce in 14-15)."""
    out = np.zeros(16, dtype=np.uint32)
    lib().oracle_chacha_block(_key_words(key).ctypes.data, counter, nonce, rounds, out.ctypes.data)
    return out


def prng_coeffs(key: bytes, nonce: int, elem_offset: int, n: int, tm1: int, rounds: int = 20) -> np.ndarray:
    """dn_m521_split_prng's coefficients of elements elem_offset..+n: uint32 [n, tm1, 17]."""
    out = np.zeros((n, tm1, 17), dtype=np.uint32)
    if n and tm1:
        lib().oracle_prng_coeffs(_key_words(key).ctypes.data, nonce, rounds, elem_offset, n, tm1, out.ctypes.data)
    return out


def mt_words(seed: int, n: int) -> np.ndarray:
    out = np.zeros(n, dtype=np.uint32)
    lib().oracle_mt_words(seed, n, out.ctypes.data)
    return out


def split(secrets: np.ndarray, coeffs: np.ndarray, t: int, n_shares: int) -> np.ndarray:
    """secrets int64 [n], coeffs uint32 [n, t-1, 17] -> shares uint32 [n_shares, n, 17]."""
    sec = np.ascontiguousarray(secrets).view(np.uint64)
    n = sec.shape[0]
    cof = np.ascontiguousarray(coeffs, dtype=np.uint32)
    out = np.zeros((n_shares, n, 17), dtype=np.uint32)
    lib().oracle_split(sec.ctypes.data, cof.ctypes.data if cof.size else None, n, t, n_shares, out.ctypes.data)
    return out


def reconstruct(ys: np.ndarray, xs) -> np.ndarray:
    """ys uint32 [k, n, 17], xs k small ints -> uint32 [n, 17]."""
    ys = np.ascontiguousarray(ys, dtype=np.uint32)
    k, n = ys.shape[0], ys.shape[1]
    xa = np.array(xs, dtype=np.int64)
    out = np.zeros((n, 17), dtype=np.uint32)
    lib().oracle_reconstruct(ys.ctypes.data, xa.ctypes.data, k, n, out.ctypes.data)
    return out
