"""fix_precision / unfix_precision (reference: delta_node/utils/precision.py:5-15).

fix_precision(arr, p)   = int64(float64(arr) * 10^p)   (C truncation; NaN and
                          out-of-range values -> INT64_MIN as numpy's x86 cast)
unfix_precision(arr, p) = float64(arr) / 10^p
Computed on the GPU (dn_bounded_i64_accumulate with no generators, and
dn_unfix_precision); numpy arrays in, numpy arrays out, like the reference.
"""
from __future__ import annotations

import numpy as np

from ..crypto.shamir import _native
from . import _mask_native as mn
from .mask import bounded_sum


def fix_precision(arr, precision: int):
    import torch

    dev = _native.require_device()
    is_np = isinstance(arr, np.ndarray)
    t = torch.as_tensor(np.asarray(arr) if not isinstance(arr, torch.Tensor) else arr)
    shape = tuple(t.shape)
    x = t.to(dev).to(torch.float64).reshape(-1).contiguous()
    out = bounded_sum([], x.numel(), 0, 2 ** 47 - 1, base_f64=x, precision=int(precision), device=dev)
    out = out.reshape(shape)
    return out.cpu().numpy() if is_np or not isinstance(arr, torch.Tensor) else out


def unfix_precision(arr, precision: int):
    import torch

    dev = _native.require_device()
    is_np = not isinstance(arr, torch.Tensor)
    t = torch.as_tensor(np.asarray(arr) if is_np else arr)
    shape = tuple(t.shape)
    if t.dtype == torch.int64:
        x = t.to(dev).reshape(-1).contiguous()
        out = torch.empty(x.numel(), dtype=torch.float64, device=dev)
        mn.unfix(x, out, x.numel(), int(precision))
    else:  # float inputs: the same IEEE float64 division, through torch on the device
        out = t.to(dev).to(torch.float64).reshape(-1) / float(10 ** int(precision))
    out = out.reshape(shape)
    return out.cpu().numpy() if is_np else out
