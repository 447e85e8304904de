#!/usr/bin/env python3
"""Codec A/B: encode / decode share x=3 of 2^24 elements, kernel time by HIP
events around the C calls (buffers preallocated), product library vs tuning
variants (CODEC_VARIANTS="DN_DECODE_W4=1;..."); one JSON line."""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "delta-node_amd"), ROOT]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from delta_node.crypto import shamir  # noqa: E402
from delta_node.crypto.shamir import _native, codec, field  # noqa: E402

N = 1 << int(os.environ.get("LOG2N", "24"))
dev = torch.device("cuda", 0)
ss = shamir.SecretShare(3)
ss.random.seed(5)
blk = ss.make_shares_vec(torch.from_numpy(np.random.default_rng(3).integers(-2**62, 2**62, N, dtype=np.int64)), 5)
vec = blk[2]
packed, offs = codec.encode_share_vec(vec, N, 3)
torch.cuda.synchronize()


def timed(reps=10):
    L = codec._lib()
    cap = int(L.dn_m521_encoded_capacity(N, 3))
    out = torch.empty(cap, dtype=torch.uint8, device=dev)
    o2 = torch.empty(N + 1, dtype=torch.int64, device=dev)
    sb = int(L.dn_m521_codec_scratch_bytes(N))
    scratch = torch.empty(sb, dtype=torch.uint8, device=dev)
    dvec = torch.empty(field.vec_bytes(N), dtype=torch.uint8, device=dev)
    xs = torch.empty(N, dtype=torch.int64, device=dev)
    bad = torch.zeros(1, dtype=torch.int32, device=dev)
    st = _native.stream_ptr()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)

    def enc():
        _native.check(L.dn_m521_encode_shares(vec.data_ptr(), N, 3, o2.data_ptr(), out.data_ptr(), cap,
                                              scratch.data_ptr(), sb, st))

    def dec():
        _native.check(L.dn_m521_decode_shares(packed.data_ptr(), packed.numel(), offs.data_ptr(), N, dvec.data_ptr(),
                                              xs.data_ptr(), bad.data_ptr(), st))

    res = {}
    for name, fn in (("encode", enc), ("decode", dec)):
        fn()
        s.record()
        for _ in range(reps):
            fn()
        e.record()
        torch.cuda.synchronize()
        res[name + "_ms"] = s.elapsed_time(e) / reps
    res["decode_equal"] = bool(torch.equal(dvec[: field.vec_bytes(N)], vec[: field.vec_bytes(N)])) and int(bad.item()) == 0
    res["encode_equal"] = bool(torch.equal(o2, offs)) and bool(torch.equal(out[: packed.numel()], packed))
    return res


out = {"product": timed()}
for var in [v for v in os.environ.get("CODEC_VARIANTS", "DN_DECODE_W4=1").split(";") if v]:
    kv = dict(x.split("=") for x in var.split(","))
    os.environ.update(kv)
    with _native.library(_native.TUNING_LIB):
        out[var] = timed()
    for k in kv:
        del os.environ[k]
print(json.dumps(out))
