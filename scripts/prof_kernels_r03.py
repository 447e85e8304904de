#!/usr/bin/env python3
"""A short run of one kernel family for rocprofv3 counter passes (round 3):
  aes   -> encrypt_vec(hex=True) of a 1.13 GB message (the bench's share
           envelope row: encrypt_kernel<14, 4, true>), 3 launches
  prng  -> split_prng ChaCha20, 3-of-5, 2^24 (split_prng_kernel<3,false>), 3 launches
  prng8 -> the same with ChaCha8 (its write floor)
  msv   -> make_shares_vec(2^24, 5) on SecretShare(3): the fused MT19937 draw +
           split (mt_jump_kernel levels, mt_gen_kernel<3>), 3 calls
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "delta-node_amd"))

import torch  # noqa: E402

what = sys.argv[1] if len(sys.argv) > 1 else "aes"
dev = torch.device("cuda", 0)
g = torch.Generator(device=dev)
g.manual_seed(1)
if what == "aes":
    from delta_node.crypto import aes

    data = torch.randint(0, 256, (1132427034,), dtype=torch.uint8, device=dev, generator=g)
    for _ in range(3):
        aes.encrypt_vec(bytes(range(32)), data, nonce=bytes(range(16, 32)), hex=True)
elif what == "msv":
    from delta_node.crypto import shamir
    from delta_node.crypto.shamir import field

    n = 1 << 24
    sec = torch.randint(-(1 << 62), 1 << 62, (n,), dtype=torch.int64, device=dev, generator=g)
    sh = torch.empty((5, field.vec_bytes(n)), dtype=torch.uint8, device=dev)
    ss = shamir.SecretShare(3)
    ss.random.seed(3)
    for _ in range(3):
        ss.make_shares_vec(sec, 5, out=sh)
else:
    from delta_node.crypto.shamir import _native, field

    n = 1 << 24
    sec = torch.randint(-(1 << 62), 1 << 62, (n,), dtype=torch.int64, device=dev, generator=g)
    sh = torch.empty((5, field.vec_bytes(n)), dtype=torch.uint8, device=dev)
    for _ in range(3):
        _native.split_prng(sec, bytes(range(32)), 0, 8 if what == "prng8" else 20, 0, sh, n, 3, 5)
torch.cuda.synchronize()
print("ok", what)
