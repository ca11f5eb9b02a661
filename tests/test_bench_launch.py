"""bench.py --gpus N without a launcher starts its own N ranks.

The driver's command shape is `python3 bench.py --gpus N`; without torchrun that process has
WORLD_SIZE unset and, before r04, measured ONE rank.  bench.launch_ranks() must run
`python -m torch.distributed.run --nproc-per-node N ... bench.py ...` as a child process before
any GPU call, relay rank 0's JSON line and return the child's exit code (CPU test: the child is
faked)."""
import io
import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


class _FakeProc:
    def __init__(self, cmd, lines, rc):
        self.cmd = cmd
        self.stdout = io.StringIO("".join(lines))
        self._rc = rc

    def wait(self):
        return self._rc


def _args(gpus):
    import argparse
    return argparse.Namespace(gpus=gpus)


def test_launch_ranks_spawns_torchrun_child(monkeypatch, capsys):
    import subprocess
    import torch
    import bench
    seen = {}
    line = json.dumps({"metric": "env-steps/sec (1024x1024, 24-plane)", "value": 1.0, "n_gpus": 8,
                       "ranks_seen": [[r, 8, r, "nccl"] for r in range(8)]})

    def fake_popen(cmd, **kw):
        seen["cmd"] = cmd
        seen["kw"] = kw
        return _FakeProc(cmd, ["RCCL version banner\n", line + "\n", "other\n"], 0)

    def no_gpu(*a, **k):
        raise AssertionError("the launcher touched the GPU before starting the ranks")

    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.setattr(subprocess, "Popen", fake_popen)
    monkeypatch.setattr(torch.cuda, "is_available", no_gpu)
    monkeypatch.setattr(torch.cuda, "init", no_gpu)
    monkeypatch.setattr(torch.cuda, "set_device", no_gpu)
    rc = bench.launch_ranks(_args(8), ["--gpus", "8", "--steps", "20"])
    assert rc == 0
    cmd = seen["cmd"]
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=8" in cmd and "--nnodes=1" in cmd and "--master-addr=127.0.0.1" in cmd
    assert any(c.startswith("--master-port=") for c in cmd)
    assert cmd[-4:] == ["--gpus", "8", "--steps", "20"]
    assert os.path.samefile(cmd[-5], os.path.join(ROOT, "bench.py"))
    out = capsys.readouterr()
    assert out.out.strip().splitlines() == [line]          # exactly rank 0's JSON line on stdout
    assert "RCCL version banner" in out.err and "other" in out.err


def test_launch_ranks_relays_failure_and_missing_line(monkeypatch):
    import subprocess
    import bench
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.setattr(subprocess, "Popen", lambda cmd, **kw: _FakeProc(cmd, ["boom\n"], 3))
    assert bench.launch_ranks(_args(2), ["--gpus", "2"]) == 3
    monkeypatch.setattr(subprocess, "Popen", lambda cmd, **kw: _FakeProc(cmd, [], 0))
    assert bench.launch_ranks(_args(2), ["--gpus", "2"]) == 1     # rc 0 but no JSON line: a failure


@pytest.mark.parametrize("gpus,world", [(1, None), (8, "8"), (2, "2")])
def test_launch_ranks_runs_in_process_when_ranked(monkeypatch, gpus, world):
    import subprocess
    import bench

    def boom(*a, **k):
        raise AssertionError("must not spawn")
    monkeypatch.setattr(subprocess, "Popen", boom)
    if world is None:
        monkeypatch.delenv("WORLD_SIZE", raising=False)
    else:
        monkeypatch.setenv("WORLD_SIZE", world)
    assert bench.launch_ranks(_args(gpus), []) is None
