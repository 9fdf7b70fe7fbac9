"""bench.py's rank launch (VERDICT r4 "next" 2): `--gpus N` runs N ranks, one process per GPU.

The decision is host logic taken before anything touches the GPU (bench.rank_launch), so it is
checked here on the CPU: no launcher and N > 1 -> a torch.distributed.run command for N ranks on
127.0.0.1 that passes the arguments through; N = 1, or a launcher's WORLD_SIZE equal to N -> run in
this process; a WORLD_SIZE that differs from N -> a non-zero exit before any work."""
import subprocess
import sys

import pytest

import bench


def test_single_gpu_runs_in_process():
    assert bench.rank_launch(["--steps", "3"], 1, {}) is None


def test_n_gpus_without_launcher_starts_n_ranks():
    argv = ["--gpus", "4", "--steps", "7", "--warmup", "2"]
    cmd = bench.rank_launch(argv, 4, {}, port=29555)
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=4" in cmd and "--nnodes=1" in cmd and "--master-port=29555" in cmd
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert cmd[-len(argv) - 1].endswith("bench.py") and cmd[-len(argv):] == argv


def test_launcher_rank_runs_in_process():
    assert bench.rank_launch(["--gpus", "2"], 2, {"WORLD_SIZE": "2", "RANK": "1"}) is None


def test_world_size_mismatch_is_an_error():
    with pytest.raises(SystemExit) as e:
        bench.rank_launch(["--gpus", "4"], 4, {"WORLD_SIZE": "2"})
    assert "WORLD_SIZE" in str(e.value)


def test_mismatch_exits_nonzero_from_the_command_line():
    """The whole script, as the driver would start it under a wrong launcher: non-zero status,
    nothing on stdout (no JSON line), before any GPU work."""
    r = subprocess.run([sys.executable, bench.__file__, "--gpus", "2"], capture_output=True, text=True,
                       env={"WORLD_SIZE": "3", "PATH": "/usr/bin:/bin"}, timeout=300)
    assert r.returncode != 0 and r.stdout.strip() == "", (r.returncode, r.stdout, r.stderr[-500:])
    assert "WORLD_SIZE" in r.stderr
