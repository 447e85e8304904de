"""Multi-rank product path on the GPU (BASELINE config 4), and config 4 at
full size on one GPU.

Two (or three) fresh child processes, gloo backend, every rank on cuda:0
(tests/gpu_dist_worker.py): `dist.draw_coeffs_sharded` (each rank jumps to its
shard of the reference's MT19937 coefficient stream and draws it on the GPU),
the HIP split of the shard, `dist.allgather_share_blocks`, and each rank's
reconstruct of its shard from the gathered vectors.  Checked against the
reference's own 5-of-9 split digest at 2^16 (tests/golden/manifest.json,
`split_t5n9_2e16`, per element shamir.py:55-66), against the unsharded
single-process split for ragged sizes, and every rank's random.Random against
the one-stream state.
"""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest
import torch

from delta_node.crypto import shamir
from delta_node.crypto.shamir import field
from golden.fixtures import manifest, secrets_int64
from oracle import c_oracle

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _start_ranks(world, args, backend, tmp_path, attempt):
    port = _free_port()
    procs, logs = [], []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), LOCAL_RANK=str(r), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), DN_DIST_BACKEND=backend)
        log = tmp_path / f"rank{r}.{attempt}.err"
        logs.append(log)
        with open(log, "w") as f:
            procs.append(subprocess.Popen([sys.executable, "-u", os.path.join(HERE, "gpu_dist_worker.py"), *args],
                                          env=env, stderr=f))
    return procs, logs


def run_ranks(world, N, t, n, mt_seed, sec_seed, tmp_path, backend="gloo"):
    """The ranks as child processes on a free port; a start that lost the
    port to another process (EADDRINUSE: the port is free when picked, not
    reserved) is started again on a new one, at most three times."""
    import time

    out = str(tmp_path / "res.json")
    args = [out, str(N), str(t), str(n), str(mt_seed), str(sec_seed)]
    for attempt in range(3):
        procs, logs = _start_ranks(world, args, backend, tmp_path, attempt)
        lost_port = False
        try:
            deadline = time.monotonic() + 100
            while any(p.poll() is None for p in procs) and time.monotonic() < deadline:
                if any(p.poll() not in (None, 0) and "EADDRINUSE" in open(lg).read() for p, lg in zip(procs, logs)):
                    lost_port = True
                    break
                time.sleep(0.2)
        finally:
            for p in procs:
                if p.poll() is None:
                    p.kill()
                    p.wait()
        if not lost_port:
            break
    for lg in logs:
        sys.stderr.write(open(lg).read())
    assert [p.returncode for p in procs] == [0] * world
    res = []
    for r in range(world):
        with open(f"{out}.{r}") as f:
            res.append(json.load(f))
    return res


def test_config4_two_ranks_equal_reference_digest(tmp_path):
    d = [d for d in manifest()["digests"] if d["name"] == "split_t5n9_2e16"][0]
    res = run_ranks(2, d["N"], d["t"], d["n"], d["mt_seed"], d["secret_seed"], tmp_path)
    assert res[0]["digest"] == d["digest"]
    assert res[0]["block_equal_single"]
    for r in res:
        assert r["device_draw"] and r["state_equal"] and r["roundtrip"], r


def test_config4_rccl_branch_world1_equal_reference_digest(tmp_path):
    """dist.py's RCCL branch on hardware: a fresh rank with
    init_process_group("nccl") on cuda:0 (world size 1 — the box has one GPU)
    runs draw_coeffs_sharded (its rejection flag all-reduced on the device),
    the HIP split and allgather_share_blocks with device tensors (no host
    staging); the gathered 5-of-9 block's digest is the reference's."""
    d = [d for d in manifest()["digests"] if d["name"] == "split_t5n9_2e16"][0]
    res = run_ranks(1, d["N"], d["t"], d["n"], d["mt_seed"], d["secret_seed"], tmp_path, backend="nccl")[0]
    assert res["backend"] == "nccl"
    assert res["via_host"] is False and res["gathered_on_device"] is True
    assert res["digest"] == d["digest"]
    assert res["block_equal_single"] and res["device_draw"] and res["state_equal"] and res["roundtrip"], res


@pytest.mark.parametrize("world,N,t,n", [(2, 65536 + 300, 5, 9), (3, 100001, 3, 5)])
def test_sharded_ranks_ragged_equal_unsharded(world, N, t, n, tmp_path):
    res = run_ranks(world, N, t, n, 99, 7, tmp_path)
    assert res[0]["block_equal_single"]
    for r in res:
        assert r["device_draw"] and r["state_equal"] and r["roundtrip"], r


@pytest.mark.slow
@pytest.mark.timeout(900)
def test_config4_full_size_one_gpu_roundtrip():
    """5-of-9 split of 2^26 int64 elements on one GPU (BASELINE config 4's
    total, unsharded) with the reference's coefficient stream: reconstruct from
    two 5-subsets equals the secrets everywhere, and ALL 2^26 elements of all
    9 shares equal the C oracle's split of the same coefficients (chunks of
    2^18 elements on 16 host threads; ctypes drops the GIL)."""
    import concurrent.futures as cf

    N, t, n = 1 << 26, 5, 9
    dev = torch.device("cuda", 0)
    sec_h = secrets_int64(26, N)
    sec = torch.from_numpy(sec_h).to(dev)
    ss = shamir.SecretShare(t)
    ss.random.seed(26)
    coeffs = ss.draw_coeffs_vec(N, dev)
    shares = torch.empty((n, field.vec_bytes(N)), dtype=torch.uint8, device=dev)
    from delta_node.crypto.shamir import _native

    _native.split_u64(sec, coeffs, shares, N, t, n)
    for xs in ([1, 3, 5, 7, 9], [2, 4, 6, 8, 9]):
        res, over = ss.resolve_shares_vec([shares[x - 1] for x in xs], xs, N, return_overflow=True)
        assert torch.equal(res, sec), xs
        assert int(over.item()) == 0
        del res

    C = 1 << 18
    nb = field.vec_bytes(C)

    def check(e0, co_b, sh_b):
        co = np.stack([field.vec_to_limbs(co_b[j], C) for j in range(t - 1)], axis=1)
        want = c_oracle.split(sec_h[e0:e0 + C], co, t, n)
        got = np.stack([field.vec_to_limbs(sh_b[x], C) for x in range(n)])
        return bool(np.array_equal(got, want))

    bad, pending = [], []
    with cf.ThreadPoolExecutor(16) as ex:
        for e0 in range(0, N, C):
            b0 = (e0 // field.TILE) * field.TILE_BYTES
            fut = ex.submit(check, e0, coeffs[:, b0:b0 + nb].cpu().numpy(), shares[:, b0:b0 + nb].cpu().numpy())
            pending.append((e0, fut))
            if len(pending) >= 32:
                e, f = pending.pop(0)
                if not f.result():
                    bad.append(e)
        for e, f in pending:
            if not f.result():
                bad.append(e)
    assert not bad, f"chunks differing from the C oracle: {bad[:8]}"
