"""fpmMain CLI contract (fpmMain.cpp:500-592): usage, device selection,
end-to-end reconstruction of a synthetic on-disk dataset.

The CPU tests check the argv / use_cpu.sh contract without touching a GPU;
the GPU test runs the whole drop-in (JSON + TIFF loader + solver + .npy and
result.json outputs) and compares with the oracle run on the same stack.
"""
import json
import os
import subprocess

import numpy as np
import pytest

from dataset_fixture import make_dataset

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "fpm-opencv_amd", "bin", "fpmMain")


def _run(args, env=None, timeout=300):
    e = dict(os.environ)
    e.pop("OPENCV_OPENCL_DEVICE", None)
    e.update(env or {})
    return subprocess.run([BIN] + args, capture_output=True, text=True, env=e, timeout=timeout)


def test_usage_without_arguments_returns_zero():
    r = _run([])
    assert r.returncode == 0
    assert "Usage" in r.stdout


def test_use_cpu_sh_device_is_refused(tmp_path):
    ds = make_dataset(str(tmp_path))
    r = _run([ds["json"], "1"], env={"OPENCV_OPENCL_DEVICE": "CPU"})
    assert r.returncode == 3
    assert "MI355X" in r.stderr


@pytest.mark.parametrize("value", ["CPU:0", ":CPU:0", "AMD Accelerated Parallel Processing:CPU:1", "cpu", ":GPU|CPU:0"])
def test_opencl_cpu_selections_are_refused(tmp_path, value):
    ds = make_dataset(str(tmp_path))
    r = _run([ds["json"], "1"], env={"OPENCV_OPENCL_DEVICE": value})
    assert r.returncode == 3, (value, r.stdout, r.stderr)


@pytest.mark.parametrize("value,extra,ordinal", [
    ("GPU:0", [], 0),                 # use_gpu.sh as shipped
    ("GPU:1", [], 1),
    (":GPU:2", [], 2),                # OpenCV's <platform>:<type>:<device>
    ("AMD:GPU:3", [], 3),
    (":GPU:", [], 0),
    ("GPU:1", ["--device", "4"], 4),  # --device wins
])
def test_opencl_gpu_index_selects_ordinal(tmp_path, value, extra, ordinal):
    # no dataset directory: the run stops at the loader, after the device line
    r = _run([str(tmp_path / "missing.json"), "1"] + extra, env={"OPENCV_OPENCL_DEVICE": value})
    assert f"Device: MI355X ordinal {ordinal}" in r.stdout.splitlines(), (value, r.stdout)
    assert r.returncode == 1


def test_grid_option_is_validated(tmp_path):
    r = _run([str(tmp_path / "missing.json"), "1", "--grid", "0x3"])
    assert r.returncode == 2 and "GXxGY" in r.stderr


@pytest.mark.gpu
def test_cli_grid_stitched_field_matches_oracle(tmp_path):
    """fpmMain --grid 2x2: four patches cut on the GPU from every full frame
    (fpm_upload_frames), solved in one batch, stitched into one field.  Each
    tile must match the host front-end's single-crop load at that patch's
    cropX/cropY run through the oracle."""
    from fpm_amd import host
    from fpm_oracle import rel_l2, run_fpm
    ds = make_dataset(str(tmp_path / "data"))
    out = tmp_path / "out"
    out.mkdir()
    r = _run([ds["json"], "2", "--out", str(out), "--grid", "2x2"], env={"OPENCV_OPENCL_DEVICE": "GPU:0"})
    assert r.returncode == 0, r.stdout + r.stderr
    meta = json.loads((out / "result.json").read_text())
    assert meta["grid"]["patches"] == 4 and meta["device"] == 0
    field = np.load(out / "objCrop_field.npy")
    pupils = np.load(out / "pupils.npy")
    k = ds["keys"]
    L = meta["nlarge"]
    Np = meta["np"]
    assert field.shape == (2 * L, 2 * L) and field.dtype == np.complex64
    assert pupils.shape == (4, Np, Np)
    for b in range(4):
        i, j = divmod(b, 2)
        d = host.Dataset(ds["json"])
        d.override("cropX", k["cropX"] + j * Np)
        d.override("cropY", k["cropY"] + i * Np)
        d.scan()
        n = d.geometry()
        d.load_images()
        cfg = d.config()
        x0, y0 = d.crops()
        ref = run_fpm(d.stack(), np.arange(n), x0, y0, cfg.np, cfg.nlarge, cfg.na_radius, cfg.delta1, cfg.delta2, 2)
        tile = field[i * L:(i + 1) * L, j * L:(j + 1) * L]
        assert rel_l2(tile, ref["objCrop"]) < 5e-5, b
        assert rel_l2(pupils[b], ref["pupil"]) < 5e-5, b


@pytest.mark.gpu
def test_cli_end_to_end_matches_oracle(tmp_path):
    from fpm_amd import host
    from fpm_oracle import rel_l2, run_fpm
    ds = make_dataset(str(tmp_path / "data"))
    out = tmp_path / "out"
    out.mkdir()
    r = _run([ds["json"], "2", "--out", str(out)], env={"OPENCV_OPENCL_DEVICE": ":GPU:0"})
    assert r.returncode == 0, r.stderr
    assert "Iteration 2 Completed" in r.stdout and "FP Processing Completed" in r.stdout
    meta = json.loads((out / "result.json").read_text())
    # the same stack and geometry through the host front-end and the oracle
    d = host.Dataset(ds["json"])
    d.scan()
    n = d.geometry()
    d.load_images()
    cfg = d.config()
    x0, y0 = d.crops()
    assert meta["leds_used"] == n and meta["order"] == d.order().tolist()
    ref = run_fpm(d.stack(), np.arange(n), x0, y0, cfg.np, cfg.nlarge, cfg.na_radius, cfg.delta1, cfg.delta2, 2)
    objcrop = np.load(out / "objCrop.npy")
    pupil = np.load(out / "pupil.npy")
    assert objcrop.shape == (cfg.nlarge, cfg.nlarge) and objcrop.dtype == np.complex64
    assert rel_l2(objcrop, ref["objCrop"]) < 5e-5
    assert rel_l2(np.load(out / "objF.npy"), ref["objF"]) < 5e-5
    assert rel_l2(pupil, ref["pupil"]) < 5e-5
