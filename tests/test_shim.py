"""Reference-side binding (include/fpm_shim.hpp) on a mock
FPM_Dataset with the reference's real layout: imageStack indexed by LED
number with ledCount+1 slots, slot 0 a dummy, unused LEDs left as the CV_8UC1
zero image with garbage crops (fpmMain.cpp:42,52-57,171).

The geometry is dataset_dogStomach.json as the reference's own jsoncpp
parses it (tests/golden/geometry_dogStomach_literal.json): ledCount 508,
157 LEDs used in the tie-ordered std::sort order, Np 200, L 600, naRadius 26,
delta1/delta2 10/3.  tests/shim/mock_runfpm.cpp drives the shim exactly as the
reference's runFPM body would; its outputs are compared with the C++ fp64
oracle on the same compacted stack.
"""
import json
import os
import struct
import subprocess

import numpy as np
import pytest

from fpm_oracle import rel_l2

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "fpm-opencv_amd", "bin", "mock_runfpm")
FIX = os.path.join(ROOT, "tests", "golden", "geometry_dogStomach_literal.json")


def _geometry():
    d = json.load(open(FIX))
    p = d["probe"]
    leds = {l["led"]: l for l in p["leds"]}
    order = p["sorted_indices"]
    x0 = np.array([leds[n]["crop_x0"] for n in order], np.int16)
    y0 = np.array([leds[n]["crop_y0"] for n in order], np.int16)
    return d["keys"], p, np.array(order, np.int16), x0, y0


def _write_input(path, p, keys, order, x0, y0, stack, itr):
    with open(path, "wb") as f:
        f.write(struct.pack("<5i", p["np"], p["nlarge"], p["led_count"], len(order), itr))
        f.write(np.array([keys["objectiveNA"], p["ps_eff"], keys["lambda"], p["delta1"], p["delta2"]],
                         np.float32).tobytes())
        f.write(order.astype("<i2").tobytes())
        f.write(x0.astype("<i2").tobytes())
        f.write(y0.astype("<i2").tobytes())
        f.write(np.ascontiguousarray(stack, "<u2").tobytes())


def test_mock_binary_built():
    assert os.path.exists(BIN), "bin/mock_runfpm missing: make -C fpm-opencv_amd"


def test_shim_refuses_8bit_slot_before_any_device_call(tmp_path):
    """A used LED whose slot still holds the CV_8UC1 dummy is refused by the
    copy adapter (no row over-read, no device call: runs without a GPU)."""
    keys, p, order, x0, y0 = _geometry()
    Np = p["np"]
    stack = np.zeros((len(order), Np, Np), np.uint16)
    inp = tmp_path / "in.bin"
    _write_input(inp, p, keys, order, x0, y0, stack, 1)
    r = subprocess.run([BIN, str(inp), str(tmp_path), "--corrupt"], capture_output=True, text=True, timeout=60)
    assert r.returncode == 4, r.stdout + r.stderr
    assert f"image of LED {int(order[3])} is not a 16-bit" in r.stdout
    assert "naRadius 26" in r.stdout
    assert not (tmp_path / "objCrop.npy").exists()


@pytest.mark.gpu
def test_shim_on_reference_layout_matches_oracle(tmp_path):
    import oracle_lib
    from tools.synth import make_stack
    keys, p, order, x0, y0 = _geometry()
    Np, L, r = p["np"], p["nlarge"], p["na_radius"]
    assert (Np, L, r, len(order), p["led_count"]) == (200, 600, 26, 157, 508)
    itr = 2
    stack = make_stack(Np, L, r, x0, y0, n_patch=1, seed=501)[:, 0]
    inp = tmp_path / "in.bin"
    _write_input(inp, p, keys, order, x0, y0, stack, itr)
    res = subprocess.run([BIN, str(inp), str(tmp_path)], capture_output=True, text=True, timeout=300)
    assert res.returncode == 0, res.stdout + res.stderr
    lines = res.stdout.splitlines()
    assert "naRadius 26" in lines
    for i in range(1, itr + 1):
        assert any(l.startswith(f"Iteration {i} Completed (Time: ") for l in lines), res.stdout
    assert lines[-1].startswith("FP Processing Completed (Time: ")
    ref = oracle_lib.run_fpm(stack, np.arange(len(order)), x0, y0, Np, L, r, p["delta1"], p["delta2"], itr)
    for k in ("objCrop", "objF", "pupil"):
        got = np.load(tmp_path / f"{k}.npy")
        assert got.dtype == np.complex128 and got.shape == ref[k].shape
        e = rel_l2(got, ref[k])
        assert e < 5e-5, (k, e)
    # pupilSupport: un-centred support disk (fpmMain.cpp:306-313), imag 0
    k = np.fft.fftfreq(Np, 1.0 / Np)
    disk = (k[:, None] ** 2 + k[None, :] ** 2) <= r * r
    sup = np.load(tmp_path / "pupilSupport.npy")
    np.testing.assert_array_equal(sup.real, disk.astype(np.float64))
    assert not sup.imag.any()
