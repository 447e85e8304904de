"""bench.py's multi-GPU entry point on the CPU: `python bench.py --gpus N`
(N > 1, no launcher environment) must run N ranks through
torch.distributed.run as a child process, and a launcher's WORLD_SIZE must
agree with --gpus.  The GPU run itself is tests/test_gpu_bench.py."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _bench():
    import importlib.util

    spec = importlib.util.spec_from_file_location("bench_mod", BENCH)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_launcher_command_runs_n_ranks_of_this_file():
    b = _bench()
    argv = ["--gpus", "8", "--steps", "5", "--warmup", "2"]
    cmd = b.launcher_cmd(8, argv, 29511)
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=8" in cmd and "--nnodes=1" in cmd
    assert "--master-addr=127.0.0.1" in cmd and "--master-port=29511" in cmd
    i = cmd.index(os.path.abspath(BENCH))
    assert cmd[i + 1:] == argv  # every rank gets the same arguments, --gpus included


def _run(args, **env):
    e = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    e.update(env)
    return subprocess.run([sys.executable, BENCH, *args], capture_output=True, text=True, env=e, timeout=120)


def test_parent_refuses_more_ranks_than_gpus_under_rccl():
    """No GPU here: 2 RCCL ranks cannot get a device each, so the parent stops
    before launching anything (and before any GPU call), with exit code 2."""
    r = _run(["--gpus", "2"], DN_DIST_BACKEND="nccl")
    assert r.returncode == 2, r.stderr
    assert "needs 2 visible GPUs" in r.stderr
    assert r.stdout == ""


def test_launcher_world_size_must_match_gpus():
    r = _run(["--gpus", "2"], WORLD_SIZE="3", RANK="0", LOCAL_RANK="0")
    assert r.returncode != 0
    assert "WORLD_SIZE=3" in r.stderr


@pytest.mark.parametrize("argv", [["--gpus", "1"], []])
def test_one_gpu_runs_in_process(argv, monkeypatch):
    """--gpus 1 (or none) never starts a launcher."""
    b = _bench()
    called = []
    monkeypatch.setattr(b, "launch_ranks", lambda *a: called.append(a) or 0)
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.setattr(sys, "argv", ["bench.py", *argv, "--steps", "0"])
    with pytest.raises(Exception):  # proceeds to the GPU part, which needs a device
        b.main()
    assert called == []
