"""Coordinator-side sum of the members' masked results.

Reference: ServerAggregator.make_masked_results, coord/horizontal/agg.py:227-251
(and its hlr twin): a member is valid when its result has exactly the task's
aggregation variables; the valid members' int64 arrays are summed per
(variable, key) with numpy's wrapping `+=`.  Here the sums run on the GPU
(dn_i64_sum, 16 inputs per pass); across GPUs, `allreduce_sum` is one RCCL
all-reduce of the per-GPU partial sums.
"""
from __future__ import annotations

from collections import defaultdict
from typing import Dict, List, Mapping, Sequence, Tuple

from ..crypto.shamir import _native
from . import _mask_native as mn


def sum_int64(tensors: Sequence, out=None):
    """sum_j tensors[j] (int64, same shape), wrapping, on the GPU."""
    import torch

    dev = _native.require_device()
    ts = [torch.as_tensor(t).to(dev).reshape(-1).contiguous() for t in tensors]
    if not ts:
        raise ValueError("sum_int64: no inputs")
    if any(t.dtype != torch.int64 for t in ts):
        raise TypeError("sum_int64: int64 inputs (masked results)")
    n = ts[0].numel()
    if any(t.numel() != n for t in ts):
        raise ValueError("sum_int64: shape mismatch")
    shape = tuple(torch.as_tensor(tensors[0]).shape)
    if out is None:
        out = torch.empty(n, dtype=torch.int64, device=dev)
    mn.i64_sum(ts[:16], out, n)
    rest = ts[16:]
    for g in range(0, len(rest), 15):  # further inputs, 15 at a time on top of `out`
        mn.i64_sum([out] + rest[g:g + 15], out, n)
    return out.reshape(shape)


def sum_member_results(member_results: Sequence[Mapping[str, Mapping[str, object]]],
                       agg_vars: Sequence[str]) -> Tuple[List[int], Dict[str, Dict[str, object]]]:
    """Indices of the valid members and the per-(var, key) sums, as
    make_masked_results computes them (device int64 tensors)."""
    valid: List[int] = []
    groups: Dict[str, Dict[str, list]] = defaultdict(lambda: defaultdict(list))
    aset = set(agg_vars)
    for idx, res in enumerate(member_results):
        names = res.keys()
        if len(names) == len(agg_vars) and len(set(names) - aset) == 0:
            valid.append(idx)
            for var in names:
                for key, val in res[var].items():
                    groups[var][key].append(val)
    out: Dict[str, Dict[str, object]] = defaultdict(dict)
    for var, keys in groups.items():
        for key, vals in keys.items():
            out[var][key] = sum_int64(vals)
    return valid, out


def allreduce_sum(t, group=None):
    """In-place RCCL all-reduce (sum) of an int64 partial sum across ranks."""
    import torch.distributed as dist

    dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
    return t
