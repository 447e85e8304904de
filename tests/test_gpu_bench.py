"""`python3 bench.py --gpus 2` on the GPU box: the parent starts two ranks
through torch.distributed.run (gloo, both on cuda:0 — the box has one GPU;
the product backend is RCCL) and prints rank 0's one JSON line, which covers
ONE 2^20-element vector split + reconstructed over the two ranks (the
per-element work of shamir.py:55-90, sharded as dist.shard_range)."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_gpus_2_launches_two_ranks():
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["DN_DIST_BACKEND"] = "gloo"
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--log2n", "20",
                        "--rows", "0", "--config4", "0", "--config5", "0", "--cpu-budget", "0",
                        "--steps", "4", "--warmup", "1", "--placements", "2"],
                       capture_output=True, text=True, env=env, timeout=110)
    assert r.returncode == 0, r.stderr[-4000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, r.stdout
    line = json.loads(lines[0])
    assert line["n_gpus"] == 2
    assert line["config"]["elements_total"] == 1 << 20
    assert line["config"]["elements_per_gpu"] == 1 << 19
    assert line["parity"]["all_ranks_ok"] is True
    assert line["weak_scaling"]["roundtrip_all_ranks"] is True


def test_bench_under_launcher_world1_rccl():
    """torch.distributed.run with one rank: bench.py forms an RCCL process
    group (nccl) at WORLD_SIZE=1, so the sharded MT draw's device all-reduce,
    the timing / parity all-reduces and config 4's RCCL all-gather run on the
    GPU."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["DN_DIST_BACKEND"] = "nccl"
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1",
                        "--master-addr=127.0.0.1", f"--master-port={port}", os.path.join(ROOT, "bench.py"),
                        "--gpus", "1", "--log2n", "20", "--rows", "0", "--config4", "1", "--config4-log2n", "20",
                        "--config5", "0", "--cpu-budget", "0", "--steps", "2", "--warmup", "1", "--placements", "2"],
                       capture_output=True, text=True, env=env, timeout=110)
    assert r.returncode == 0, r.stderr[-4000:]
    line = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert line["n_gpus"] == 1 and line["parity"]["all_ranks_ok"] is True
    assert line["config4"]["allgather"]["blocks_equal"] is True
    assert line["config4"]["allgather"]["all_ranks_ok"] is True


def test_bench_rows_small():
    """The one-GPU bench with every §8(f) row on, at 2^18 elements: each row's
    code runs (a row that raises fails the driver's bench line) and its parity
    flags hold."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--log2n", "18", "--steps", "2",
                        "--warmup", "1", "--placements", "2", "--config4", "0", "--config5", "0",
                        "--cpu-budget", "0"],
                       capture_output=True, text=True, env=env, timeout=110)
    assert r.returncode == 0, r.stderr[-4000:]
    line = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert line["parity"]["all_ranks_ok"] is True
    rows = line["rows"]
    for k in ("share_codec", "share_envelope", "split_prng", "member_sum", "mask_masking", "draw_split", "byte_api"):
        assert k in rows, k
    assert rows["share_codec"]["roundtrip_equal"] and rows["share_codec"]["kernels_equal_api"]
    env_row = rows["share_envelope"]
    assert env_row["roundtrip_equal"] and env_row["oracle_prefix_equal"] and env_row["encrypt_kernel_equal_api"]
    assert rows["draw_split"]["equal_draw_then_split_and_state"]


@pytest.mark.timeout(400)
def test_bench_gpus_8_driver_command_rehearsal():
    """The driver's N=8 command, rehearsed with 8 gloo ranks on the box's one
    GPU at 2^20 elements: one JSON line with n_gpus 8, every rank's parity,
    config 4's all-gather checked on every rank, and the reference CPU path
    timed in the same run (cpu_baseline at every world size)."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["DN_DIST_BACKEND"] = "gloo"
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "8", "--log2n", "20",
                        "--config4", "1", "--config4-log2n", "20", "--rows", "0", "--config5", "0",
                        "--cpu-budget", "2", "--steps", "4", "--warmup", "1", "--placements", "2"],
                       capture_output=True, text=True, env=env, timeout=380)
    assert r.returncode == 0, r.stderr[-4000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, r.stdout
    line = json.loads(lines[0])
    assert line["n_gpus"] == 8
    assert line["config"]["elements_per_gpu"] == 1 << 17
    assert line["parity"]["all_ranks_ok"] is True
    assert line["config4"]["allgather"]["all_ranks_ok"] is True
    cb = line["cpu_baseline"]
    assert cb["run_at_world_size"] == 8 and cb["value"] > 0 and cb["cores"] == 1
    assert cb["c_port"]["value"] > 0
