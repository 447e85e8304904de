"""MiMC7 commitments on the GPU.

Reference: delta_node/utils/mimc7.py:18-92, `__all__ = ["calc_weight_commitment",
"calc_data_commitment"]` (gmpy2 arithmetic over the BN254 scalar field,
utils/constant.py).  Same names, inputs and outputs; the row hashes and the
Merkle trees of calc_data_commitment run one lane per row / one workgroup per
128-row block on the GPU (dn_mimc7_data_rows, dn_mimc7_merkle_blocks); the
weight commitment is one strictly sequential chain of dependent field products
and runs natively on the calling host core (dn_mimc7_weight_commitment_host,
csrc/host_mimc7.cpp — see its header for the measured reason), exact for every
finite weight.  dn_mimc7_weight_chain is the same chain on one device lane, for
device-resident weights (weight_commitment_device).
"""
from __future__ import annotations

import ctypes
from typing import Iterable, List

import numpy as np

from .. import serialize
from ..crypto.shamir import _native

__all__ = ["calc_weight_commitment", "calc_data_commitment"]

Q = 21888242871839275222246405745257275088548364400416034343698204186575808495617
DATA_BLOCK = 128
EXPORTS = ("dn_mimc7_data_rows", "dn_mimc7_merkle_blocks", "dn_mimc7_weight_chain", "dn_mimc7_hash",
           "dn_mimc7_weight_commitment_host", "dn_mimc7_params")
def _lib():
    L = _native.lib()
    if not getattr(L, "_dn_mimc7_bound", False):  # argtypes, once per loaded library
        vp, u64, i32 = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int
        L.dn_mimc7_data_rows.restype = i32
        L.dn_mimc7_data_rows.argtypes = [vp, u64, i32, vp, vp, vp]
        L.dn_mimc7_merkle_blocks.restype = i32
        L.dn_mimc7_merkle_blocks.argtypes = [vp, u64, vp, vp]
        L.dn_mimc7_weight_chain.restype = i32
        L.dn_mimc7_weight_chain.argtypes = [vp, u64, i32, vp, vp, vp]
        L.dn_mimc7_hash.restype = i32
        L.dn_mimc7_hash.argtypes = [vp, vp, u64, vp, vp]
        L.dn_mimc7_weight_commitment_host.restype = i32
        L.dn_mimc7_weight_commitment_host.argtypes = [vp, u64, i32, vp]
        L._dn_mimc7_bound = True
    return L


def _limbs_to_int(row) -> int:
    return int.from_bytes(np.ascontiguousarray(row, dtype="<u4").tobytes(), "little")


def _ints_to_limbs(vals, width=8) -> np.ndarray:
    return np.frombuffer(b"".join(int(v).to_bytes(4 * width, "little") for v in vals), dtype="<u4").reshape(-1, width)


def _check_bad(bad) -> None:
    if int(bad.item()):
        raise NotImplementedError("mimc7: |value * 10^precision| >= 2^253 is not handled on the device")


def mimc7_hash(xs, keys) -> List[int]:
    """Batched mimc7_hash(x, key) (mimc7.py:18-27) for ints in [0, q): unreduced r + key."""
    import torch

    dev = _native.require_device()
    xs, keys = list(xs), list(keys)
    if any(not 0 <= int(v) < Q for v in xs + keys):
        raise ValueError("mimc7_hash: inputs must be in [0, q)")
    n = len(xs)
    x = torch.from_numpy(_ints_to_limbs(xs).copy()).to(dev)
    k = torch.from_numpy(_ints_to_limbs(keys).copy()).to(dev)
    out = torch.empty((n, 9), dtype=torch.int32, device=dev)
    _native.check(_lib().dn_mimc7_hash(x.data_ptr(), k.data_ptr(), n, out.data_ptr(), _native.stream_ptr()))
    return [_limbs_to_int(r) for r in out.cpu().numpy().view(np.uint32)]


def data_row_hashes(data):
    """Device uint32 [round_up(rows, 128), 8] row hashes of calc_data_commitment."""
    import torch

    dev = _native.require_device()
    arr = torch.as_tensor(np.asarray(data, dtype=np.float64) if not isinstance(data, torch.Tensor) else data)
    arr = arr.to(dev).to(torch.float64).contiguous()
    rows, cols = int(arr.shape[0]), int(arr.shape[1])
    rows_pad = -(-rows // DATA_BLOCK) * DATA_BLOCK
    out = torch.empty((rows_pad, 8), dtype=torch.int32, device=dev)
    bad = torch.zeros(1, dtype=torch.int32, device=dev)
    _native.check(_lib().dn_mimc7_data_rows(arr.data_ptr(), rows, cols, out.data_ptr(), bad.data_ptr(),
                                            _native.stream_ptr()))
    _check_bad(bad)
    return out


def calc_data_commitment(data: Iterable[Iterable[float]]) -> List[bytes]:
    """mimc7.py:63-92: one commitment (minimal big-endian bytes) per 128 rows."""
    import torch

    leaves = data_row_hashes(data)
    blocks = leaves.shape[0] // DATA_BLOCK
    roots = torch.empty((blocks, 8), dtype=torch.int32, device=leaves.device)
    _native.check(_lib().dn_mimc7_merkle_blocks(leaves.data_ptr(), blocks, roots.data_ptr(), _native.stream_ptr()))
    return [serialize.int_to_bytes(_limbs_to_int(r)) for r in roots.cpu().numpy().view(np.uint32)]


def calc_weight_commitment(weight: Iterable[float]) -> bytes:
    """mimc7.py:58-60: mimc7_hash_arr([_float2mpz(w, 8) for w in weight], 2), minimal big-endian bytes.

    Weights are converted to float64 first (numpy 1.22 value-based casting makes
    the reference's float32 * 10**8 a float64 product too).  A torch tensor is
    read back to the host.  NaN raises ValueError, +-inf OverflowError, as
    int() does in the reference.
    """
    if hasattr(weight, "detach"):  # torch tensor
        weight = weight.detach().cpu().numpy()
    w = np.ascontiguousarray(np.asarray(weight if isinstance(weight, np.ndarray) else list(weight),
                                        dtype=np.float64).reshape(-1))
    out = (ctypes.c_uint32 * 8)()
    _native.check(_lib().dn_mimc7_weight_commitment_host(w.ctypes.data if w.size else None, w.size, 8,
                                                         ctypes.addressof(out)))
    return serialize.int_to_bytes(int.from_bytes(bytes(out), "little"))


def weight_commitment_device(weight) -> bytes:
    """The same chain on one device lane (dn_mimc7_weight_chain) for a device float64 tensor.

    Latency-bound (one dependent product at a time on one lane): slower than
    calc_weight_commitment's host chain; |w * 10^8| >= 2^253 raises
    NotImplementedError.
    """
    import torch

    dev = _native.require_device()
    if not isinstance(weight, torch.Tensor):  # lists would otherwise become float32 tensors
        weight = torch.from_numpy(np.asarray(weight, dtype=np.float64).reshape(-1).copy())
    w = weight.to(dev).to(torch.float64).contiguous().reshape(-1)
    out = torch.empty(8, dtype=torch.int32, device=dev)
    bad = torch.zeros(1, dtype=torch.int32, device=dev)
    _native.check(_lib().dn_mimc7_weight_chain(w.data_ptr(), w.numel(), 8, out.data_ptr(), bad.data_ptr(),
                                               _native.stream_ptr()))
    _check_bad(bad)
    return serialize.int_to_bytes(_limbs_to_int(out.cpu().numpy().view(np.uint32)))
