"""bench.py's launcher contract on the CPU (no GPU call is reached):
`--gpus N` without a launcher re-launches itself under torch.distributed.run
with N ranks (one per GPU) as a child process and exits with its status; under
a launcher whose WORLD_SIZE differs from --gpus it refuses to run.  A 1-GPU
number must never be labelled N GPUs (round-2 review)."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run_main(monkeypatch, argv, env):
    import bench
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        monkeypatch.delenv(k, raising=False)
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    monkeypatch.setattr(sys, "argv", ["bench.py"] + argv)
    calls = []
    import subprocess
    monkeypatch.setattr(subprocess, "call", lambda cmd, *a, **k: calls.append(cmd) or 7)
    with pytest.raises(SystemExit) as e:
        bench.main()
    return e.value.code, calls


def test_gpus_n_spawns_one_rank_per_gpu(monkeypatch):
    code, calls = _run_main(monkeypatch, ["--gpus", "8", "--steps", "3", "--warmup", "1"], {})
    assert code == 7 and len(calls) == 1              # the child's exit status is returned
    cmd = calls[0]
    assert cmd[1:3] == ["-m", "torch.distributed.run"]
    assert "--nproc-per-node=8" in cmd and "127.0.0.1" in cmd
    assert cmd[-6:] == ["--gpus", "8", "--steps", "3", "--warmup", "1"]


def test_gpus_mismatch_under_launcher_refuses(monkeypatch):
    code, calls = _run_main(monkeypatch, ["--gpus", "8"], {"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    assert calls == [] and "WORLD_SIZE=2" in str(code)
