"""Shamir secret sharing over GF(2^521 - 1) — the `delta_node.crypto.shamir` surface.

Drop-in for delta_node/crypto/shamir/shamir.py (same names, arguments, return
values and exceptions), backed by the MI355X HIP library through its C-ABI
(`_native`, include/dn_shamir.h):

=============================  =============================================
reference (shamir.py)          here
=============================  =============================================
``Share``, ``PRIME`` :14-16    same objects
``_eval_at`` :19-25            device Horner (`dn_m521_split_fe`)
``_share_to_bytes`` :28-33     same codec (host, per share)
``_bytes_to_share`` :36-45     same codec (host, per share)
``SecretShare.__init__`` :49   same attributes: threshold, prime, random
``make_shares`` :55-66         coefficients from ``self.random`` exactly as
                               the reference draws them; evaluation in the
                               library's host path (one secret per call)
``resolve_shares`` :68-90      same checks/messages/exceptions, library host
                               path (any prime)
=============================  =============================================

Vector extension (the hot path, new): ``make_shares_vec`` splits a whole
int64 tensor, element e behaving exactly like
``make_shares(v_e.to_bytes(8, "big", signed=True), n)`` called in order on the
same instance; ``resolve_shares_vec`` interpolates whole share vectors.

There is no CPU fallback: without the native library every call raises, and
without a HIP device every vector call raises.  The byte API (one secret per
call, as the reference's callers use it) runs in the library's native host
path (csrc/host_shamir.cpp) for any prime, like the reference's
``SecretShare(t, prime=q)``; the vector API is GF(2^521 - 1) on the GPU.
"""
from __future__ import annotations

import random
from functools import reduce
from typing import List, Optional, Sequence, Tuple, Union

from ... import serialize
from . import _native, field, memory, op

__all__ = ["Share", "PRIME", "SecretShare"]

Share = Tuple[int, int]

PRIME = (1 << 521) - 1  # 0x01FF...FF, the Mersenne prime M521 (shamir.py:16)


# ------------------------------------------------------------------ codec
def _share_to_bytes(share: Share) -> bytes:
    """``[len(x) as 1 byte][x minimal BE][y minimal BE]`` (shamir.py:28-33)."""
    x, y = share
    xb = serialize.int_to_bytes(x)
    return len(xb).to_bytes(1, "big") + xb + serialize.int_to_bytes(y)


def _bytes_to_share(data: bytes) -> Share:
    """Inverse of `_share_to_bytes` (shamir.py:36-45)."""
    xl = int.from_bytes(data[:1], "big")
    return serialize.bytes_to_int(data[1:1 + xl]), serialize.bytes_to_int(data[1 + xl:])


# ------------------------------------------------------- device helpers
def _device():
    _native.lib()
    return _native.require_device()


def _to_device_vecs(ints: Sequence[int], dev):
    """Python ints (each < 2^521) -> uint8 device tensor [len, vec_bytes(1)]."""
    import numpy as np
    import torch

    host = np.stack([field.ints_to_vec([v]) for v in ints]) if ints else np.zeros((0, field.vec_bytes(1)), np.uint8)
    return torch.from_numpy(host).to(dev)


def _device_values(values, dev, name: str):
    """`values` as a contiguous 1-D int64 tensor on `dev` (no conversion when
    it already is one: the common call, a resident vector)."""
    import torch

    if (isinstance(values, torch.Tensor) and values.device == dev and values.dtype == torch.int64
            and values.dim() == 1 and values.is_contiguous()):
        return values
    vals = torch.as_tensor(values)
    if vals.dtype not in (torch.int64, torch.uint64):
        raise TypeError(f"{name}: values must be an int64 tensor")
    return vals.reshape(-1).to(dev).contiguous()


def _eval_many(coeffs: Sequence[int], n_shares: int) -> List[int]:
    """y(x) = sum_j coeffs[j] x^j mod p for x = 1..n_shares, on the GPU.
    coeffs[0] is the secret (any size; reduced mod p here)."""
    import torch

    dev = _device()
    t = len(coeffs)
    sec = _to_device_vecs([coeffs[0] % PRIME], dev)
    cof = _to_device_vecs(list(coeffs[1:]), dev) if t > 1 else None
    out = torch.empty((n_shares, field.vec_bytes(1)), dtype=torch.uint8, device=dev)
    _native.split_fe(sec, cof, out, 1, t, n_shares)
    host = out.cpu().numpy()
    return [field.vec_to_ints(host[i], 1)[0] for i in range(n_shares)]


def _eval_at(coeffs: List[int], x: int, prime: int) -> int:
    """Horner evaluation of `coeffs` at x mod prime (shamir.py:19-25).

    GF(2^521 - 1) with 1 <= x <= 65535 and at most 64 coefficients runs the
    device split (`dn_m521_split_fe`); every other input — another prime
    (negative too), x = 0, a negative or larger x, more coefficients — runs
    the library's host Horner (`dn_shamir_eval_at_host`), which computes
    exactly what the reference's loop computes for any integers."""
    if not coeffs:
        return 0
    if prime == PRIME and 1 <= x <= _native.MAX_SHARES and len(coeffs) <= _native.MAX_THRESHOLD:
        return _eval_many([c % prime for c in coeffs], x)[x - 1]
    return _native.host_eval_at([int(c) for c in coeffs], int(x), int(prime))


def _draw_coeffs_generic(rng, n: int, tm1: int):
    """The reference's own draw for a generator that is not plain MT19937
    (random.SystemRandom, a subclass overriding randint / getrandbits ...):
    `rng.randint(1, p - 1)` per coefficient, element-major (shamir.py:59-61),
    packed as a host block [tm1, vec_bytes(n)]."""
    import numpy as np

    cols = [[0] * n for _ in range(tm1)]
    for e in range(n):
        for j in range(tm1):
            cols[j][e] = rng.randint(1, PRIME - 1)
    return np.stack([field.ints_to_vec(c) for c in cols])


def _lagrange_generic(xs: Sequence[int], prime: int) -> List[int]:
    """lambda_i = prod_{j!=i} (-x_j) / prod_{j!=i} (x_i - x_j) mod p, as the
    reference forms nums/dens (shamir.py:77-83) and divides (op.py:28-29)."""
    k = len(xs)
    lams = []
    for i in range(k):
        num = reduce(lambda a, b: a * b, [-xs[j] for j in range(k) if j != i])
        den = reduce(lambda a, b: a * b, [xs[i] - xs[j] for j in range(k) if j != i])
        lams.append(op.div_mod(num % prime, den, prime))
    return lams


def _resolve_vectors(vecs: Sequence, xs: Sequence[int], n: int, threshold: int,
                     out_fe=None, out_u64=None, overflow=None) -> None:
    """Lagrange-at-0 of device share vectors `vecs` (abscissas xs) into
    out_fe / out_u64, on the GPU.  k <= 16 with 64-bit xs uses the native
    small-rational weights; otherwise full-width weights in groups of 16 whose
    partial vectors are then summed mod p on the device."""
    import torch

    k = len(xs)
    if k <= _native.MAX_RESOLVE and all(0 <= int(x) < (1 << 64) for x in xs):
        w = _native.lagrange(xs, threshold)
        _native.reconstruct(vecs, w, out_fe=out_fe, out_u64=out_u64, overflow=overflow, n=n)
        return
    lams = _lagrange_generic([int(x) for x in xs], PRIME)
    vb = field.vec_bytes(n)
    dev = vecs[0].device
    G = _native.MAX_RESOLVE
    parts = []
    for g in range(0, k, G):
        part = torch.empty(vb, dtype=torch.uint8, device=dev)
        _native.reconstruct(vecs[g:g + G], _native.generic_weights(lams[g:g + G]), out_fe=part, n=n)
        parts.append(part)
    while len(parts) > G:  # sum partial vectors mod p, 16 at a time
        merged = []
        for g in range(0, len(parts), G):
            dst = torch.empty(vb, dtype=torch.uint8, device=dev)
            _native.reconstruct(parts[g:g + G], _native.ones_weights(len(parts[g:g + G])), out_fe=dst, n=n)
            merged.append(dst)
        parts = merged
    _native.reconstruct(parts, _native.ones_weights(len(parts)), out_fe=out_fe, out_u64=out_u64,
                        overflow=overflow, n=n)


# ------------------------------------------------------------------ API
class SecretShare(object):
    """Threshold-`threshold` Shamir scheme over GF(PRIME) (shamir.py:48-90)."""

    def __init__(self, threshold: int, *, prime: int = PRIME):
        self.threshold = threshold
        self.prime = prime
        self.random = random.Random()
        self.last_draw_rejected = False

    def _require_m521(self):
        if self.prime != PRIME:
            raise NotImplementedError("the vector (GPU) path is GF(2^521 - 1) only; the byte API takes any prime")

    # ---- reference byte API -------------------------------------------
    def make_shares(self, value: bytes, shares: int) -> List[bytes]:
        """Split `value` into `shares` byte shares (shamir.py:55-66).

        One secret per call — the reference's callers' pattern — so the field
        arithmetic runs in the library's host path (dn_shamir_make_shares_host:
        a GPU launch and two copies would cost ~20x the reference's latency);
        the coefficients are drawn from `self.random` exactly as the reference
        draws them."""
        if self.threshold > shares:
            raise ValueError("threshold should be little equal than shares")
        serialize.bytes_to_int(value)  # the reference's conversion (and its errors)
        coeffs = [self.random.randint(1, self.prime - 1) for _ in range(self.threshold - 1)]
        if shares <= 0:
            return []
        return _native.host_make_shares(bytes(value), coeffs, self.prime, self.threshold, shares)

    def resolve_shares(self, shares: List[bytes]) -> bytes:
        """Recover the secret from byte shares (shamir.py:68-90): the
        Lagrange interpolant of ALL given shares at 0, minimal big-endian, with
        the reference's checks and messages (dn_shamir_resolve_shares_host)."""
        shares = [bytes(s) for s in shares]
        if not shares:  # zip(*[]) unpacked into xs, ys
            raise ValueError("not enough values to unpack (expected 2, got 0)")
        return _native.host_resolve_shares(shares, self.threshold, self.prime)

    # ---- vector extension (the hot path) -------------------------------
    def draw_coeffs_vec(self, n: int, device=None, *, elem_offset: int = 0, n_total: Optional[int] = None):
        """The (t-1) x n coefficients that n sequential `make_shares` calls
        would draw from `self.random` (advancing it identically), as a uint8
        device tensor [t-1, vec_bytes(n)] in the tiled layout.

        Sharded form (elem_offset / n_total): the coefficients of elements
        [elem_offset, elem_offset + n) of an n_total-element draw — the words
        before the shard are skipped by jump-ahead (dn_mt19937_skip) — and
        `self.random` ends as after the whole n_total-element draw.  Exact
        unless a 521-bit draw is rejected (odds ~2^-520 each) in the skipped
        range; `self.last_draw_rejected` reports one in this shard's range, and
        `dist.draw_coeffs_sharded` combines the flags over ranks."""
        self._require_m521()
        import torch

        dev = device if device is not None else _device()
        tm1 = max(self.threshold, 1) - 1
        sharded = elem_offset != 0 or (n_total is not None and n_total != n)
        if not _native.mt_compatible(self.random):
            # not CPython's MT19937 draw: call it, as the reference does
            if sharded:
                raise NotImplementedError("draw_coeffs_vec: a sharded draw needs a plain random.Random "
                                          f"(jump-ahead), not {type(self.random).__name__}")
            self.last_draw_rejected = False
            if tm1 <= 0 or n <= 0:
                return torch.zeros((max(tm1, 0), field.vec_bytes(n)), dtype=torch.uint8, device=dev)
            return torch.from_numpy(_draw_coeffs_generic(self.random, n, tm1)).to(dev)
        if sharded:
            if n_total is None or not 0 <= elem_offset <= elem_offset + n <= n_total:
                raise ValueError("draw_coeffs_vec: shard [elem_offset, elem_offset + n) must lie in [0, n_total)")
            rng = random.Random()
            rng.setstate(self.random.getstate())
            _native.mt_skip(rng, 17 * tm1 * elem_offset)
        else:
            rng = self.random
        self.last_draw_rejected = False
        blk = None
        if tm1 > 0 and n > 0 and torch.device(dev).type == "cuda":
            # bit-exact MT19937 on the GPU (jump-ahead substreams); the host
            # draw below is the fallback for a rejected draw (odds ~2^-520)
            vb = field.vec_bytes(n)
            # a share-block allocation (memory.py): the split reads it at 2 x 66 B per
            # element; 1-2 % faster from a probed 2 MiB-chunk block (profiles/r04/p/)
            blk = memory.share_block((tm1, vb), dev)
            if n % field.TILE:
                blk[:, vb - field.TILE_BYTES:].zero_()  # padding lanes of the last tile, as the host draw leaves them
            if not _native.mt_draw_coeffs_device(rng, n, tm1, blk):
                blk = None
        if blk is None:
            probe = random.Random()
            probe.setstate(rng.getstate())
            host = _native.mt_draw_coeffs(rng, n, tm1)
            _native.mt_skip(probe, 17 * tm1 * n)
            self.last_draw_rejected = probe.getstate() != rng.getstate()  # a rejection consumed extra words
            blk = torch.from_numpy(host).to(dev)
        if sharded:
            _native.mt_skip(self.random, 17 * tm1 * n_total)
        return blk

    def make_shares_vec(self, values, shares: int, *, coeffs=None, out=None):
        """Split every element of an int64 tensor.

        values  int64 tensor [N] (any device; copied to the current HIP device)
        coeffs  optional uint8 device tensor [t-1, vec_bytes(N)]; default: drawn
                from `self.random` as N sequential `make_shares` calls would
        out     optional uint8 device tensor [shares, vec_bytes(N)]; default: a
                pooled block of 16 MiB physical chunks (memory.share_block)
        Returns uint8 device tensor [shares, vec_bytes(N)]: row x-1 holds share x
        of every element (tiled M521 layout, canonical residues).
        """
        self._require_m521()
        import torch

        if self.threshold > shares:
            raise ValueError("threshold should be little equal than shares")
        if shares > _native.MAX_SHARES or self.threshold > _native.MAX_THRESHOLD:
            raise NotImplementedError("make_shares_vec: at most 65535 shares and threshold 64")
        dev = _device()
        vals = _device_values(values, dev, "make_shares_vec")
        n = vals.numel()
        t = max(self.threshold, 1)
        vb = field.vec_bytes(n)
        if out is None:  # pooled chunked block (memory.py: the split's fast placement)
            out = memory.share_block((max(shares, 0), vb), dev)
        elif (out.dtype != torch.uint8 or tuple(out.shape) != (shares, vb) or not out.is_contiguous()
              or out.device != dev):
            raise ValueError(f"make_shares_vec: out must be contiguous uint8 [{shares}, {vb}] on {dev}")
        if (coeffs is None and t > 1 and n > 0 and shares > 0 and _native.mt_compatible(self.random)
                and _native.mt_split_device(self.random, vals, out, n, t, shares)):
            # fused: the reference's MT19937 draws feed the split in registers (no coefficient block)
            self.last_draw_rejected = False
            return out
        if coeffs is None:
            coeffs = self.draw_coeffs_vec(n, dev) if t > 1 else None
        elif t > 1:
            if coeffs.dtype != torch.uint8 or tuple(coeffs.shape) != (t - 1, vb) or coeffs.device != dev:
                raise ValueError(f"make_shares_vec: coeffs must be uint8 [{t - 1}, {vb}] on {dev}")
            coeffs = coeffs.contiguous()
        if shares > 0:
            _native.split_u64(vals, coeffs if t > 1 else None, out, n, t, shares)
        return out

    def make_shares_vec_prng(self, values, shares: int, *, key: Optional[bytes] = None, nonce: int = 0,
                             rounds: int = 20, elem_offset: int = 0, out=None):
        """Split every element with coefficients generated on the device.

        Same shares layout as `make_shares_vec`, but the coefficients come from
        a keyed ChaCha stream (dn_m521_split_prng) instead of `self.random`:
        each is uniform in [1, p-1] and depends only on (key, nonce, global
        element index elem_offset + e), so sharded calls reproduce the
        unsharded result.  key: 32 bytes (default: fresh from `secrets`);
        rounds: 20 (default), 12 or 8.  Returns (shares block, key).
        """
        self._require_m521()
        import secrets as _secrets

        import torch

        if self.threshold > shares:
            raise ValueError("threshold should be little equal than shares")
        if shares > _native.MAX_SHARES or self.threshold > 8:
            raise NotImplementedError("make_shares_vec_prng: at most 65535 shares and threshold 8")
        if key is None:
            key = _secrets.token_bytes(32)
        dev = _device()
        vals = _device_values(values, dev, "make_shares_vec_prng")
        n = vals.numel()
        vb = field.vec_bytes(n)
        if out is None:
            out = memory.share_block((max(shares, 0), vb), dev)
        elif (out.dtype != torch.uint8 or tuple(out.shape) != (shares, vb) or not out.is_contiguous()
              or out.device != dev):
            raise ValueError(f"make_shares_vec_prng: out must be contiguous uint8 [{shares}, {vb}] on {dev}")
        if shares > 0:
            if self.threshold <= 1:
                _native.split_u64(vals, None, out, n, 1, shares)
            else:
                _native.split_prng(vals, key, nonce, rounds, elem_offset, out, n, self.threshold, shares)
        return out, key

    def resolve_shares_vec(self, shares, xs: Sequence[int], n: int, *, out: str = "int64",
                           return_overflow: bool = False):
        """Interpolate share vectors at 0 (vector form of `resolve_shares`).

        shares  sequence of k uint8 device tensors [vec_bytes(n)] (or a [k, vec_bytes(n)] tensor)
        xs      their abscissas (share x of `make_shares_vec` is row x-1)
        out     "int64": int64 tensor [n] holding the low 64 bits (the secret's
                two's-complement view); "field": uint8 tiled vector [vec_bytes(n)]
        return_overflow  also return a uint32 device counter of elements >= 2^64
        Same checks as `resolve_shares` (too few, duplicates, k == 1).
        """
        self._require_m521()
        import torch

        vecs = list(shares.unbind(0)) if isinstance(shares, torch.Tensor) and shares.dim() == 2 else list(shares)
        xs = [int(x) for x in xs]
        if len(vecs) != len(xs):
            raise ValueError("resolve_shares_vec: one abscissa per share vector")
        if len(xs) == 0:
            raise ValueError("not enough values to unpack (expected 2, got 0)")
        k = len(xs)
        if k < self.threshold:
            raise ValueError("need at least {} shares".format(self.threshold))
        if k != len(set(xs)):
            raise ValueError("shares must be distinct")
        if k == 1:
            raise TypeError("reduce() of empty iterable with no initial value")
        dev = _device()
        vb = field.vec_bytes(n)
        for v in vecs:
            if v.dtype != torch.uint8 or v.numel() != vb or v.device != dev or not v.is_contiguous():
                raise ValueError(f"resolve_shares_vec: share vectors must be contiguous uint8 [{vb}] on {dev}")
        over = torch.zeros(1, dtype=torch.int32, device=dev) if return_overflow else None
        if out == "int64":
            res = torch.empty(n, dtype=torch.int64, device=dev)
            _resolve_vectors(vecs, xs, n, self.threshold, out_u64=res, overflow=over)
        elif out == "field":
            res = torch.empty(vb, dtype=torch.uint8, device=dev)
            _resolve_vectors(vecs, xs, n, self.threshold, out_fe=res, overflow=over)
        else:
            raise ValueError('resolve_shares_vec: out must be "int64" or "field"')
        return (res, over) if return_overflow else res
