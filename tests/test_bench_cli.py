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


def test_general_path_traffic_counts_every_patch_group(tmp_path):
    """The general path runs each per-LED kernel once per patch group, so a
    counter file's per-dispatch bytes cover one group: bench.load_pmc scales
    them by the kernel's dispatches over the profiled run's LED steps (the
    rounds 5-6 config 5 figure of 2.80x was one group's)."""
    import json
    import bench
    from tools.srchash import src_hash
    per = {"k_rows256_inv": 1.0e6, "k_cols256": 2.0e6, "k_rows256_fwd": 3.0e6, "k_pupil_commit": 0.5e6}
    disp = {"k_rows256_inv": 386, "k_cols256": 386, "k_rows256_fwd": 386, "k_pupil_commit": 2}
    p = tmp_path / "pmc.json"
    p.write_text(json.dumps({"src_hash": src_hash(), "per_launch_hbm_bytes": per, "dispatches": disp,
                             "derived": {}}))
    tot, _, note = bench.load_pmc(str(p), "general_led_step", n_led=193)
    assert tot == pytest.approx(2 * (1.0e6 + 2.0e6 + 3.0e6) + 0.5e6 * 2 / 193)
    assert "dispatches" in note
    # a file without dispatch counts (older tools) keeps the one-group sum and says so
    p.write_text(json.dumps({"src_hash": src_hash(), "per_launch_hbm_bytes": per, "derived": {}}))
    tot, _, note = bench.load_pmc(str(p), "general_led_step", n_led=193)
    assert tot == pytest.approx(6.5e6) and "one patch group" in note
    # a fused kernel: one dispatch per iteration, the per-dispatch bytes as they are
    p.write_text(json.dumps({"src_hash": src_hash(), "per_launch_hbm_bytes": {"k_fused_s90": 4.0e8},
                             "dispatches": {"k_fused_s90": 1}, "derived": {}}))
    tot, _, _ = bench.load_pmc(str(p), "k_fused_s90", n_led=193)
    assert tot == 4.0e8
