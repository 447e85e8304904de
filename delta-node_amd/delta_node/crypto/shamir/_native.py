"""ctypes binding of the C-ABI library `libdn_shamir.so` (include/dn_shamir.h).

The product path is the HIP library: there is no CPU fallback.  If the
library is missing, or no HIP device is visible when a device call is made,
these helpers raise instead of computing anything on the host.

torch is imported before the library is loaded so that the library's
`libamdhip64.so.7` dependency resolves to the HIP runtime torch already
loaded (same soname), i.e. one runtime, one set of streams per process.
"""
from __future__ import annotations

import array
import contextlib
import ctypes
import os
import threading
from typing import List, Optional, Sequence

import numpy as np

DN_OK = 0
DN_ERR_ARG = -1
DN_ERR_THRESHOLD = -2
DN_ERR_TOO_FEW = -3
DN_ERR_DISTINCT = -4
DN_ERR_HIP = -5
DN_ERR_UNSUPPORTED = -6
DN_ERR_EMPTY = -7
DN_ERR_RETRY = -8
DN_ERR_ZERODIV = -9
DN_ERR_ASSERT = -10
DN_ERR_OVERFLOW = -11

MAX_RESOLVE = 16
MAX_THRESHOLD = 64
MAX_SHARES = 65535

_HERE = os.path.dirname(os.path.abspath(__file__))
DEFAULT_LIB = os.path.normpath(os.path.join(_HERE, "..", "..", "..", "lib", "libdn_shamir.so"))

# Every symbol include/dn_shamir.h declares (checked by the CPU test suite).
EXPORTS = (
    "dn_m521_vec_bytes", "dn_m521_split_u64", "dn_m521_split_fe", "dn_m521_lagrange",
    "dn_m521_reconstruct", "dn_mt19937_draw_coeffs", "dn_last_error", "dn_version",
    "dn_m521_split_prng", "dn_m521_prng_coeffs",
    "dn_mt19937_device_scratch_bytes", "dn_mt19937_draw_coeffs_device", "dn_mt19937_skip",
    "dn_mt19937_split_device", "dn_mt19937_split_supported", "dn_shamir_make_shares_host", "dn_shamir_resolve_shares_host",
    "dn_shamir_eval_at_host", "dn_block_granularity", "dn_block_alloc", "dn_block_free", "dn_block_probe_rows",
    "dn_block_record", "dn_block_ready", "dn_block_acquire", "dn_block_retired_bytes",
    "dn_mt19937_rt_rows_embedded", "dn_mt19937_spec_stats", "dn_mt19937_jump_poly",
)


class Lagrange(ctypes.Structure):
    """Mirror of dn_m521_lagrange_t."""

    _fields_ = [
        ("k", ctypes.c_int32),
        ("a_limbs", ctypes.c_int32),
        ("neg", ctypes.c_uint32),
        ("shift", ctypes.c_int32),
        ("has_inv", ctypes.c_int32),
        ("d", ctypes.c_uint32),
        ("a", (ctypes.c_uint32 * 17) * MAX_RESOLVE),
        ("inv", ctypes.c_uint32 * 17),
        ("d_inv32", ctypes.c_uint32),
        ("p_inv_d", ctypes.c_uint32),
        ("d_recip", ctypes.c_uint64),
        ("w", ctypes.c_uint32 * 17),
        ("reserved", ctypes.c_uint32),
    ]


_lock = threading.Lock()
_lib: Optional[ctypes.CDLL] = None


def lib_path() -> str:
    return os.environ.get("DN_SHAMIR_LIB", DEFAULT_LIB)


def lib() -> ctypes.CDLL:
    """Load (once) and return the native library; raise if it is missing."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is None:
            _lib = _load(lib_path())
        return _lib


@contextlib.contextmanager
def library(path: str):
    """Bind another build of the same C-ABI for the duration of a block —
    the tuning build (lib/libdn_shamir_tuning.so, whose DN_* knobs select
    kernel variants) in the variant-equivalence tests.  Not thread-safe; the
    product library is restored on exit."""
    global _lib
    prev = lib()
    with _lock:
        _lib = _load(path)
    try:
        yield _lib
    finally:
        with _lock:
            _lib = prev


TUNING_LIB = os.path.join(os.path.dirname(DEFAULT_LIB), "libdn_shamir_tuning.so")


def _load(path: str) -> ctypes.CDLL:
    import torch  # noqa: F401  (bind the HIP runtime torch already loaded)

    if not os.path.exists(path):
        raise RuntimeError(
            f"libdn_shamir.so not found at {path}: build it with `make -C delta-node_amd` "
            "(or __graft_entry__.build()); the Shamir hot path has no CPU fallback")
    L = ctypes.CDLL(path)
    vp, u64, i32 = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int
    L.dn_m521_vec_bytes.restype = u64
    L.dn_m521_vec_bytes.argtypes = [u64]
    L.dn_m521_split_u64.restype = i32
    L.dn_m521_split_u64.argtypes = [vp, vp, vp, u64, i32, i32, vp]
    L.dn_m521_split_fe.restype = i32
    L.dn_m521_split_fe.argtypes = [vp, vp, vp, u64, i32, i32, vp]
    L.dn_m521_lagrange.restype = i32
    L.dn_m521_split_prng.restype = i32
    L.dn_m521_split_prng.argtypes = [vp, vp, u64, i32, u64, vp, u64, i32, i32, vp]
    L.dn_m521_prng_coeffs.restype = i32
    L.dn_m521_prng_coeffs.argtypes = [vp, u64, i32, u64, vp, u64, i32, vp]
    L.dn_m521_lagrange.argtypes = [ctypes.POINTER(ctypes.c_uint64), i32, i32, ctypes.POINTER(Lagrange)]
    L.dn_m521_reconstruct.restype = i32
    L.dn_m521_reconstruct.argtypes = [ctypes.POINTER(vp), ctypes.POINTER(Lagrange), vp, vp, vp, u64, vp]
    L.dn_mt19937_draw_coeffs.restype = i32
    L.dn_mt19937_draw_coeffs.argtypes = [ctypes.POINTER(ctypes.c_uint32), ctypes.POINTER(ctypes.c_int32), u64,
                                         i32, vp]
    L.dn_mt19937_device_scratch_bytes.restype = u64
    L.dn_mt19937_device_scratch_bytes.argtypes = [u64, i32]
    L.dn_mt19937_draw_coeffs_device.restype = i32
    L.dn_mt19937_draw_coeffs_device.argtypes = [vp, vp, u64, i32, vp, vp, u64, vp]  # state, index by address
    L.dn_mt19937_split_device.restype = i32
    L.dn_mt19937_split_device.argtypes = [vp, vp, vp, vp, u64, i32, i32, vp, u64, vp]
    L.dn_mt19937_split_supported.restype = i32
    L.dn_mt19937_split_supported.argtypes = [u64, i32, i32]
    L.dn_shamir_make_shares_host.restype = i32
    L.dn_shamir_make_shares_host.argtypes = [ctypes.c_char_p, u64, ctypes.c_char_p, ctypes.c_uint32, i32,
                                             ctypes.c_char_p, ctypes.c_uint32, u64, vp, u64, vp]
    L.dn_shamir_resolve_shares_host.restype = i32
    L.dn_shamir_resolve_shares_host.argtypes = [ctypes.c_char_p, vp, i32, i32, ctypes.c_char_p, ctypes.c_uint32, vp,
                                                u64, ctypes.POINTER(ctypes.c_uint64)]
    L.dn_shamir_eval_at_host.restype = i32
    L.dn_shamir_eval_at_host.argtypes = [ctypes.c_char_p, vp, ctypes.c_char_p, i32, ctypes.c_char_p,
                                         ctypes.c_uint32, i32, ctypes.c_char_p, ctypes.c_uint32, i32, vp, u64,
                                         ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_int)]
    L.dn_block_granularity.restype = i32
    L.dn_block_granularity.argtypes = [i32, ctypes.POINTER(ctypes.c_uint64)]
    L.dn_block_alloc.restype = i32
    L.dn_block_alloc.argtypes = [u64, u64, i32, ctypes.POINTER(ctypes.c_void_p)]
    L.dn_block_free.restype = i32
    L.dn_block_free.argtypes = [vp]
    L.dn_block_record.restype = i32
    L.dn_block_record.argtypes = [vp, vp]
    L.dn_block_ready.restype = i32
    L.dn_block_ready.argtypes = [vp, vp, ctypes.POINTER(ctypes.c_int)]
    L.dn_block_acquire.restype = i32
    L.dn_block_acquire.argtypes = [vp, vp, i32]
    L.dn_mt19937_rt_rows_embedded.restype = i32
    L.dn_mt19937_rt_rows_embedded.argtypes = []
    if hasattr(L, "dn_mt19937_spec_stats"):  # (an A/B baseline built from an older revision may lack these)
        L.dn_mt19937_spec_stats.restype = i32
        L.dn_mt19937_spec_stats.argtypes = [ctypes.POINTER(u64)]
    if hasattr(L, "dn_mt19937_jump_poly"):
        L.dn_mt19937_jump_poly.restype = i32
        L.dn_mt19937_jump_poly.argtypes = [u64, ctypes.POINTER(u64)]
    L.dn_block_retired_bytes.restype = i32
    L.dn_block_retired_bytes.argtypes = [ctypes.POINTER(ctypes.c_uint64)]
    L.dn_block_probe_rows.restype = i32
    L.dn_block_probe_rows.argtypes = [vp, ctypes.c_uint32, u64, vp]
    L.dn_mt19937_skip.restype = i32
    L.dn_mt19937_skip.argtypes = [ctypes.POINTER(ctypes.c_uint32), ctypes.POINTER(ctypes.c_int32), u64]
    L.dn_last_error.restype = ctypes.c_char_p
    L.dn_last_error.argtypes = []
    L.dn_version.restype = ctypes.c_char_p
    L.dn_version.argtypes = []
    return L


def last_error() -> str:
    return lib().dn_last_error().decode()


def check(rc: int) -> None:
    """Map a DN_ERR_* code to the reference's exception type (shamir.py:57,73,75)."""
    if rc == DN_OK:
        return
    msg = last_error()
    if rc in (DN_ERR_THRESHOLD, DN_ERR_TOO_FEW, DN_ERR_DISTINCT, DN_ERR_ARG):
        raise ValueError(msg)
    if rc == DN_ERR_EMPTY:
        raise TypeError(msg)
    if rc == DN_ERR_UNSUPPORTED:
        raise NotImplementedError(msg)
    if rc == DN_ERR_ZERODIV:
        raise ZeroDivisionError(*([] if msg == "ZeroDivisionError" else [msg]))
    if rc == DN_ERR_ASSERT:
        raise AssertionError
    if rc == DN_ERR_OVERFLOW:
        raise OverflowError(msg)
    raise RuntimeError(f"dn_shamir error {rc}: {msg}")


# ------------------------------------------------------------------ device
_HAS_DEVICE = False  # a HIP device has been seen (it does not go away)


def require_device():
    """The current HIP device; raise if there is none (no CPU fallback)."""
    global _HAS_DEVICE
    import torch

    if not _HAS_DEVICE:
        if not torch.cuda.is_available():
            raise RuntimeError("delta_node.crypto.shamir: no HIP device visible; the MI355X path has no CPU fallback")
        _HAS_DEVICE = True
    return torch.device("cuda", torch.cuda.current_device())


def has_device() -> bool:
    """True when a HIP device is visible (cached once seen); never raises."""
    global _HAS_DEVICE
    if _HAS_DEVICE:
        return True
    import torch

    _HAS_DEVICE = bool(torch.cuda.is_available())
    return _HAS_DEVICE


def stream_ptr() -> int:
    """The current device's current stream (hipStream_t as an int)."""
    import torch

    return torch._C._cuda_getCurrentRawStream(torch.cuda.current_device())


def _ptr(t) -> Optional[int]:
    return None if t is None else t.data_ptr()


def vec_bytes(n: int) -> int:
    return int(lib().dn_m521_vec_bytes(n))


def split_u64(secrets, coeffs, shares, n: int, t: int, n_shares: int) -> None:
    check(lib().dn_m521_split_u64(_ptr(secrets), _ptr(coeffs), _ptr(shares), n, t, n_shares, stream_ptr()))


def split_fe(secrets_fe, coeffs, shares, n: int, t: int, n_shares: int) -> None:
    check(lib().dn_m521_split_fe(_ptr(secrets_fe), _ptr(coeffs), _ptr(shares), n, t, n_shares, stream_ptr()))


def _key_words(key: bytes):
    if not isinstance(key, (bytes, bytearray)) or len(key) != 32:
        raise ValueError("PRNG key must be 32 bytes")
    return (ctypes.c_uint32 * 8).from_buffer_copy(bytes(key))


def split_prng(secrets, key: bytes, nonce: int, rounds: int, elem_offset: int, shares, n: int, t: int,
               n_shares: int) -> None:
    check(lib().dn_m521_split_prng(_ptr(secrets), _key_words(key), nonce, rounds, elem_offset, _ptr(shares), n, t,
                                   n_shares, stream_ptr()))


def prng_coeffs(key: bytes, nonce: int, rounds: int, elem_offset: int, coeffs, n: int, tm1: int) -> None:
    check(lib().dn_m521_prng_coeffs(_key_words(key), nonce, rounds, elem_offset, _ptr(coeffs), n, tm1, stream_ptr()))


def lagrange(xs: Sequence[int], threshold: int) -> Lagrange:
    w = Lagrange()
    arr = (ctypes.c_uint64 * max(1, len(xs)))(*[int(x) for x in xs])
    check(lib().dn_m521_lagrange(arr, len(xs), threshold, ctypes.byref(w)))
    return w


def generic_weights(lams: Sequence[int]) -> Lagrange:
    """Descriptor for explicit weights lambda_i in [0, p) (full-width form)."""
    if not 1 <= len(lams) <= MAX_RESOLVE:
        raise ValueError("generic_weights: 1..16 weights")
    w = Lagrange()
    w.k = len(lams)
    w.a_limbs = 17
    for i, lam in enumerate(lams):
        for j in range(17):
            w.a[i][j] = (lam >> (32 * j)) & 0xFFFFFFFF
    return w


def ones_weights(k: int) -> Lagrange:
    """Descriptor summing k vectors mod p (all lambda_i = 1)."""
    w = Lagrange()
    w.k = k
    w.a_limbs = 1
    for i in range(k):
        w.a[i][0] = 1
    return w


def reconstruct(share_vecs: Sequence, w: Lagrange, out_fe=None, out_u64=None, overflow=None, n: int = 0) -> None:
    k = len(share_vecs)
    if k != w.k:
        raise ValueError("reconstruct: weight/share count mismatch")
    ptrs = (ctypes.c_void_p * k)(*[v.data_ptr() for v in share_vecs])
    check(lib().dn_m521_reconstruct(ptrs, ctypes.byref(w), _ptr(out_fe), _ptr(out_u64), _ptr(overflow), n,
                                    stream_ptr()))


def mt_draw_coeffs(rng, n: int, tm1: int) -> np.ndarray:
    """Draw n*(t-1) coefficients from `rng` (a random.Random) exactly as n
    sequential `make_shares` calls would (shamir.py:59-61), into a host block
    of tm1 tiled vectors; `rng`'s state advances identically."""
    vb = vec_bytes(n)
    out = np.zeros(max(tm1, 0) * vb, dtype=np.uint8)
    if tm1 <= 0 or n == 0:
        return out.reshape(max(tm1, 0), vb)
    version, gauss, state, index = _mt_state(rng)
    check(lib().dn_mt19937_draw_coeffs(state, ctypes.byref(index), n, tm1, out.ctypes.data))
    _mt_set_state(rng, version, gauss, state, index)
    return out.reshape(tm1, vb)


def _mt_state(rng):
    """rng's MT19937 array as a ctypes uint32[624] (over an array.array: ~10x
    cheaper than building a ctypes array from 624 Python ints) and its index."""
    version, internal, gauss = rng.getstate()
    buf = array.array("I", internal[:624])
    return version, gauss, (ctypes.c_uint32 * 624).from_buffer(buf), ctypes.c_int32(internal[624])


def _mt_set_state(rng, version, gauss, state, index) -> None:
    rng.setstate((version, tuple(memoryview(state).cast("B").cast("I").tolist()) + (index.value,), gauss))


# CPython's random.Random keeps its MT19937 array inside the object —
# Modules/_randommodule.c: {PyObject_HEAD; int index; uint32_t state[624];},
# the same in 3.8 .. 3.12 — and a subclass instance keeps those fields at the
# same offsets.  When this interpreter's layout checks out (once, against
# getstate() of a probe, reads and a write), the device draws take pointers
# into the caller's generator and update it in place on success: no
# getstate / setstate round trip (~36 us of a ~1.5 ms 2^24 make_shares_vec
# call).  Otherwise (another interpreter, another layout) they marshal.
_MT_LAYOUT = None  # None: not checked yet; False: unavailable; else (index offset, state offset)


def _mt_layout():
    global _MT_LAYOUT
    if _MT_LAYOUT is None:
        _MT_LAYOUT = False
        try:
            import _random
            import random as _rnd
            import sys

            head = ctypes.sizeof(ctypes.c_ssize_t) + ctypes.sizeof(ctypes.c_void_p)  # ob_refcnt, ob_type
            off_i, off_s = head, head + 4
            if sys.implementation.name == "cpython" and _random.Random.__basicsize__ >= off_s + 4 * 624:
                probe = _rnd.Random(0x5EED)
                probe.getrandbits(32 * 101)  # index mid-array
                st = probe.getstate()[1]
                words = (ctypes.c_uint32 * 624).from_address(id(probe) + off_s)
                idx = ctypes.c_int32.from_address(id(probe) + off_i)
                if list(words) == list(st[:624]) and idx.value == st[624]:
                    words[7] ^= 1
                    seen = probe.getstate()[1][7]
                    words[7] ^= 1
                    if seen == st[7] ^ 1 and probe.getstate() == (3, st, None):
                        _MT_LAYOUT = (off_i, off_s)
        except Exception:  # pragma: no cover - any surprise: marshal instead
            _MT_LAYOUT = False
    return _MT_LAYOUT


# The methods through which the reference's `self.random.randint(1, p - 1)`
# (shamir.py:60) reaches the MT19937 words.  A subclass overriding any of them
# (random.SystemRandom: os.urandom; a recording or seeded-differently
# generator) draws something else, so the MT paths below must not serve it.
_MT_METHODS = ("randint", "randrange", "_randbelow", "getrandbits", "random", "getstate", "setstate", "seed")


_MT_CLASS_OK = {}  # class -> mt_compatible verdict (classes are not re-patched at run time)


def mt_compatible(rng) -> bool:
    """True when `rng.randint` is CPython's MT19937 draw: a random.Random
    whose class overrides none of the methods the draw goes through.  Only
    then may the device / host MT paths (jump-ahead, the caller's state read
    directly) replace the reference's per-coefficient calls."""
    cls = type(rng)
    ok = _MT_CLASS_OK.get(cls)
    if ok is None:
        import random as _rnd

        ok = issubclass(cls, _rnd.Random) and all(getattr(cls, m, None) is getattr(_rnd.Random, m)
                                                  for m in _MT_METHODS)
        _MT_CLASS_OK[cls] = ok
    return ok


def _mt_inplace(rng):
    """(uint32* state, int32* index) into rng's own MT19937 state, or None."""
    lay = _mt_layout()
    if not lay or not mt_compatible(rng):
        return None
    return (ctypes.cast(id(rng) + lay[1], ctypes.POINTER(ctypes.c_uint32)),
            ctypes.cast(id(rng) + lay[0], ctypes.POINTER(ctypes.c_int32)))


def _mt_inplace_addr(rng):
    """(state address, index address) inside rng's own MT19937 state, or None."""
    lay = _mt_layout()
    if not lay or not mt_compatible(rng):
        return None
    return id(rng) + lay[1], id(rng) + lay[0]


def mt_skip(rng, words: int) -> None:
    """Advance `rng` (a random.Random) by `words` 32-bit outputs by jump-ahead."""
    version, gauss, state, index = _mt_state(rng)
    check(lib().dn_mt19937_skip(state, ctypes.byref(index), int(words)))
    _mt_set_state(rng, version, gauss, state, index)


_tls = threading.local()


def _mt_scratch(nbytes: int, device):
    """The device MT draw's scratch (job tables, windows), cached per thread
    and device: every draw synchronises its stream before it returns, so the
    thread's scratch is idle between its calls (no allocation per call)."""
    import torch

    cache = getattr(_tls, "scratch", None)
    if cache is None:
        cache = _tls.scratch = {}
    buf = cache.get(device)
    if buf is None or buf.numel() < nbytes:
        cache[device] = buf = torch.empty(max(nbytes, 1 << 20), dtype=torch.uint8, device=device)
    return buf


def mt_draw_coeffs_device(rng, n: int, tm1: int, out) -> bool:
    """`mt_draw_coeffs` with the coefficients generated on the GPU into `out`
    (uint8 device tensor [tm1, vec_bytes(n)]), bit-exact; `rng` advances
    identically.  Returns False (rng untouched) when the draw must be redone on
    the host: a rejected 521-bit draw (odds ~2^-520 each) or a stream beyond
    the jump table."""
    import torch

    if tm1 <= 0 or n == 0:
        return True
    vb = vec_bytes(n)
    if out.dtype != torch.uint8 or tuple(out.shape) != (tm1, vb) or not out.is_contiguous() or not out.is_cuda:
        raise ValueError(f"mt_draw_coeffs_device: out must be a contiguous uint8 device tensor [{tm1}, {vb}]")
    L = lib()
    sb = int(L.dn_mt19937_device_scratch_bytes(n, tm1))
    scratch = _mt_scratch(sb, out.device)
    ip = _mt_inplace_addr(rng)  # the entry point writes the state only on success
    if ip:
        rc = L.dn_mt19937_draw_coeffs_device(ip[0], ip[1], n, tm1, out.data_ptr(), scratch.data_ptr(), sb,
                                             stream_ptr())
    else:
        version, gauss, state, index = _mt_state(rng)
        rc = L.dn_mt19937_draw_coeffs_device(ctypes.addressof(state), ctypes.addressof(index), n, tm1,
                                             out.data_ptr(), scratch.data_ptr(), sb, stream_ptr())
    if rc in (DN_ERR_RETRY, DN_ERR_UNSUPPORTED):
        return False
    check(rc)
    if not ip:
        _mt_set_state(rng, version, gauss, state, index)
    return True


_MT_SPLIT_SHAPES: dict = {}  # (library, n, t, n_shares) -> (fused split supported, scratch bytes)


def mt_split_device(rng, secrets, shares, n: int, t: int, n_shares: int) -> bool:
    """make_shares over n int64 secrets with coefficients drawn from `rng`
    (a random.Random) as n sequential make_shares calls would, draw and split
    fused on the GPU (dn_mt19937_split_device) into `shares` (uint8 device
    [n_shares, vec_bytes(n)]).  False (rng untouched, shares unspecified) when
    the fused form does not apply or a draw was rejected: draw, then split."""
    import torch

    if n == 0:
        return True
    L = lib()
    key = (id(L), n, t, n_shares)
    shape = _MT_SPLIT_SHAPES.get(key)  # (supported, scratch bytes): two C calls per new shape only
    if shape is None:
        sup = bool(L.dn_mt19937_split_supported(n, t, n_shares))
        shape = (sup, int(L.dn_mt19937_device_scratch_bytes(n, t - 1)) if sup else 0)
        if len(_MT_SPLIT_SHAPES) >= 256:
            _MT_SPLIT_SHAPES.clear()
        _MT_SPLIT_SHAPES[key] = shape
    if not shape[0]:
        return False  # before any allocation: the draw, then the split
    for name, x in (("secrets", secrets), ("shares", shares)):
        if not x.is_cuda or x.device != shares.device or not x.is_contiguous():
            raise ValueError(f"mt_split_device: {name} must be a contiguous tensor on the shares' HIP device")
    sb = shape[1]
    scratch = _mt_scratch(sb, shares.device)
    ip = _mt_inplace_addr(rng)  # the entry point writes the state only on success
    if ip:
        rc = L.dn_mt19937_split_device(ip[0], ip[1], secrets.data_ptr(), shares.data_ptr(), n, t, n_shares,
                                       scratch.data_ptr(), sb, stream_ptr())
    else:
        version, gauss, state, index = _mt_state(rng)
        rc = L.dn_mt19937_split_device(ctypes.addressof(state), ctypes.addressof(index), secrets.data_ptr(),
                                       shares.data_ptr(), n, t, n_shares, scratch.data_ptr(), sb, stream_ptr())
    if rc in (DN_ERR_RETRY, DN_ERR_UNSUPPORTED):
        return False
    check(rc)
    if not ip:
        _mt_set_state(rng, version, gauss, state, index)
    return True


def mt_jump_poly(words: int):
    """x^words mod P as 312 little-endian uint64 words (dn_mt19937_jump_poly)."""
    import numpy as np

    out = (ctypes.c_uint64 * 312)()
    check(lib().dn_mt19937_jump_poly(words, out))
    return np.frombuffer(out, dtype=np.uint64).copy()


def mt_spec_stats() -> dict:
    """The current device's draw speculation counters (dn_mt19937_spec_stats):
    hits, misses, launched, armed."""
    out = (ctypes.c_uint64 * 4)()
    check(lib().dn_mt19937_spec_stats(out))
    return {"hits": int(out[0]), "misses": int(out[1]), "launched": int(out[2]), "armed": bool(out[3])}


# ------------------------------------------------------------------ host (byte API)
M521 = (1 << 521) - 1


def _prime_arg(prime: int):
    if prime == M521:
        return None, 0, 66
    pb = prime.to_bytes(max(1, (prime.bit_length() + 7) // 8), "big")
    return pb, len(pb), len(pb)


def host_make_shares(value: bytes, coeffs: Sequence[int], prime: int, threshold: int, n: int) -> List[bytes]:
    """The reference's make_shares arithmetic for one secret on the host
    (dn_shamir_make_shares_host, csrc/host_shamir.cpp): `value` is coefficient
    0 as the caller's bytes, `coeffs` the t-1 drawn coefficients; returns the
    n share records ([len(x)][x][y], shamir.py:28-33)."""
    pb, plen, w = _prime_arg(prime)
    cb = b"".join([c.to_bytes(w, "big") for c in coeffs])
    cap = n * (9 + w)
    out = ctypes.create_string_buffer(cap)
    offs = (ctypes.c_uint64 * (n + 1))()
    rc = (_lib or lib()).dn_shamir_make_shares_host(value, len(value), cb, w, threshold, pb, plen, n, out, cap, offs)
    if rc:
        check(rc)
    raw = ctypes.string_at(out, offs[n])
    o = offs[:]
    return [raw[o[i]:o[i + 1]] for i in range(n)]


def host_resolve_shares(shares: Sequence[bytes], threshold: int, prime: int) -> bytes:
    """The reference's resolve_shares arithmetic on the host
    (dn_shamir_resolve_shares_host): parse, checks (same messages), Lagrange
    at 0 over all k shares, minimal big-endian bytes."""
    pb, plen, w = _prime_arg(prime)
    k = len(shares)
    offs = (ctypes.c_uint64 * (k + 1))()
    o = 0
    for i, s in enumerate(shares):
        offs[i] = o
        o += len(s)
    offs[k] = o
    out = ctypes.create_string_buffer(w + 8)
    n = ctypes.c_uint64(0)
    rc = (_lib or lib()).dn_shamir_resolve_shares_host(b"".join(shares), offs, k, threshold, pb, plen, out, w + 8,
                                                       ctypes.byref(n))
    if rc:
        check(rc)
    return ctypes.string_at(out, n.value)


def _mag(v: int) -> bytes:
    v = abs(v)
    return v.to_bytes((v.bit_length() + 7) // 8, "big")


def host_eval_at(coeffs: Sequence[int], x: int, prime: int) -> int:
    """`_eval_at` (shamir.py:19-25) for any integers on the host
    (dn_shamir_eval_at_host): Horner with Python's `% prime` after each step."""
    k = len(coeffs)
    mags = [_mag(c) for c in coeffs]
    offs = (ctypes.c_uint64 * (k + 1))()
    o = 0
    for i, m in enumerate(mags):
        offs[i] = o
        o += len(m)
    offs[k] = o
    neg = bytes(int(c < 0) for c in coeffs)
    xb, pb = _mag(x), _mag(prime)
    cap = max(len(pb), 1) + 8
    out = ctypes.create_string_buffer(cap)
    n, sgn = ctypes.c_uint64(0), ctypes.c_int(0)
    rc = (_lib or lib()).dn_shamir_eval_at_host(b"".join(mags), offs, neg, k, xb, len(xb), int(x < 0), pb, len(pb),
                                                int(prime < 0), out, cap, ctypes.byref(n), ctypes.byref(sgn))
    if rc:
        check(rc)
    v = int.from_bytes(ctypes.string_at(out, n.value), "big")
    return -v if sgn.value else v


def version() -> str:
    return lib().dn_version().decode()


def exported_symbols() -> List[str]:
    L = lib()
    return [s for s in EXPORTS if hasattr(L, s)]
