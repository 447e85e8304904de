"""Fused secure-aggregation masking on the GPU.

Reference call pattern (runner/horizontal/agg.py:284-318, client side):

    seed_mask = make_mask(seed, shape)
    sk_mask = sum(+-make_mask(shared_key_v, shape) for v in u2 if v != self)
    masked = fix_precision(val, precision) + seed_mask + sk_mask      # int64, wraps

and its inverse on the coordinator (coord/horizontal/agg.py:381-404):
`val -= make_mask(seed)` per alive member, `val -+= make_mask(key)` per
(dead member, alive member) key, then `unfix_precision`.

`masked_sum` computes base + sum_j sign_j * make_mask(seed_j) in one pass per
16 generators (dn_bounded_i64_accumulate), bit-exact with numpy: any generator
whose raw draws hit a Lemire rejection (odds 2^-47 per element) is replayed
with the exact per-segment raw offsets numpy's sequential loop implies.
"""
from __future__ import annotations

from typing import Optional, Sequence, Tuple, Union

from ..crypto.shamir import _native
from . import _mask_native as mn

MASK_LOW, MASK_HIGH = 0, 2 ** 47 - 1  # arr.py:26: integers(0, 2**47 - 1)

Seed = Union[int, bytes]


def _replay_exact(out, g, sign: int, n: int, low: int, rng: int, dev) -> None:
    """Undo generator g's (shifted) contribution and add the exact one."""
    mn.accumulate([g], [-sign], out, n, low, rng, base_i64=out)
    slack = 64
    while True:
        cnt, rej = mn.list_rejects(g, rng, 0, n + slack, slack + 64, dev)
        if cnt <= slack:  # every raw draw an element can need (< n + cnt) was scanned
            break
        slack = 2 * cnt + 64
    # element e draws raw e + j once j rejections precede it:
    # offset j covers elements [r_j + 1 - j, r_{j+1} - j)  (r_0 - 0 + 1 := 0)
    bounds = [0] + [r + 1 - j for j, r in enumerate(rej, start=1)]
    ends = [r - j for j, r in enumerate(rej)] + [n]
    for j, (b, e) in enumerate(zip(bounds, ends)):
        b, e = max(b, 0), min(e, n)
        if e > b:
            mn.accumulate([g], [sign], out, n, low, rng, base_i64=out, raw_offsets=[j], elem_begin=b, elem_end=e)


def bounded_sum(terms: Sequence[Tuple[Seed, int]], n: int, low: int, high: int, *, base_i64=None, base_f64=None,
                precision: int = 0, out=None, device=None):
    """out[e] = base[e] + sum_j sign_j * Generator(PCG64(seed_j)).integers(low, high, n, int64)[e]."""
    import torch

    dev = device if device is not None else _native.require_device()
    rng = high - 1 - low
    if out is None:
        out = torch.empty(n, dtype=torch.int64, device=dev)
    gens = [mn.pcg64(s) for s, _ in terms]
    signs = [int(sg) for _, sg in terms]
    if any(sg not in (1, -1) for sg in signs):
        raise ValueError("signs must be +1 or -1")
    flags = torch.zeros(max(1, len(gens)), dtype=torch.int32, device=dev)
    first = True
    for i in range(0, max(1, len(gens)), mn.MAX_GENS):
        grp, sg = gens[i:i + mn.MAX_GENS], signs[i:i + mn.MAX_GENS]
        if first:
            mn.accumulate(grp, sg, out, n, low, rng, base_i64=base_i64, base_f64=base_f64, precision=precision,
                          rejects=flags[i:])
        else:
            mn.accumulate(grp, sg, out, n, low, rng, base_i64=out, rejects=flags[i:])
        first = False
    if gens:
        bad = [j for j, f in enumerate(flags[: len(gens)].cpu().tolist()) if f]
        for j in bad:
            _replay_exact(out, gens[j], signs[j], n, low, rng, dev)
    return out


def masked_sum(values, terms: Sequence[Tuple[Seed, int]], precision: Optional[int] = None, out=None):
    """fix_precision(values, precision) (if precision is given; else values is
    int64) + sum_j sign_j * make_mask(seed_j, values.shape), on the GPU."""
    import torch

    dev = _native.require_device()
    v = torch.as_tensor(values).to(dev).contiguous()
    shape = tuple(v.shape)
    n = v.numel()
    if precision is None:
        if v.dtype != torch.int64:
            raise TypeError("masked_sum: int64 values, or float values with a precision")
        res = bounded_sum(terms, n, MASK_LOW, MASK_HIGH, base_i64=v.reshape(-1), out=out)
    else:
        res = bounded_sum(terms, n, MASK_LOW, MASK_HIGH, base_f64=v.to(torch.float64).reshape(-1),
                          precision=int(precision), out=out)
    return res.reshape(shape)


def unmasked_values(masked, terms: Sequence[Tuple[Seed, int]], precision: int):
    """Coordinator side: masked + sum_j sign_j * make_mask(seed_j) (signs chosen
    by the caller, e.g. -1 per alive seed), then unfix_precision -> float64."""
    import torch

    dev = _native.require_device()
    m = torch.as_tensor(masked).to(dev).contiguous()
    ints = bounded_sum(terms, m.numel(), MASK_LOW, MASK_HIGH, base_i64=m.reshape(-1))
    out = torch.empty(m.numel(), dtype=torch.float64, device=dev)
    mn.unfix(ints, out, m.numel(), int(precision))
    return out.reshape(tuple(m.shape))
