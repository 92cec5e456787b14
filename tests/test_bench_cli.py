"""CPU: bench.py's launcher contract (no GPU needed).  ``--gpus N`` must never report a run with a
different number of ranks: without a launcher it starts N ranks itself (bench.launch_ranks), and
under a launcher whose WORLD_SIZE disagrees it exits non-zero."""
import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402


def test_world_size_mismatch_exits(monkeypatch):
    monkeypatch.setenv("WORLD_SIZE", "1")
    with pytest.raises(SystemExit, match="WORLD_SIZE=1"):
        bench.setup_dist(8, "nccl")
    monkeypatch.setenv("WORLD_SIZE", "4")
    with pytest.raises(SystemExit, match="WORLD_SIZE=4"):
        bench.setup_dist(2, "nccl")


def test_launcher_command(monkeypatch):
    seen = {}

    class R:
        returncode = 7

    def fake_run(cmd, env):
        seen["cmd"], seen["env"] = cmd, env
        return R()

    import subprocess
    monkeypatch.setattr(subprocess, "run", fake_run)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "4", "--steps", "2"])
    assert bench.launch_ranks(4) == 7
    cmd = seen["cmd"]
    assert cmd[1:3] == ["-m", "torch.distributed.run"] and "--nproc-per-node=4" in cmd
    assert "--master-addr=127.0.0.1" in cmd and cmd[-4:] == ["--gpus", "4", "--steps", "2"]
    assert seen["env"]["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"
