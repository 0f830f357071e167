"""Loader preprocessing on the GPU (fpm_upload_frames, fpmMain.cpp:124-144)
vs the oracle's numpy restatement, bit-exact (integer work), for several
patches cut from each full frame, host and device frame sources (GPU only)."""
import numpy as np
import pytest

import fpm_oracle as oracle
import fpm_amd
from tools.synth import grid_geometry

pytestmark = pytest.mark.gpu

NP, L, R = 32, 96, 6
H, W = 300, 280
PATCHES = [(0, 0), (37, 11), (248, 268), (120, 90)]   # (x0, y0): includes the frame corner
BK1, BK2 = (5, 250), (200, 3)


def _frames(n, seed=1):
    rng = np.random.default_rng(seed)
    f = rng.integers(0, 4000, (n, H, W)) + rng.integers(0, 2000, (n, 1, 1))
    f[:, 100:200, 50:150] += rng.integers(0, 60000, (n, 100, 100))   # saturating pixels
    return np.clip(f, 0, 65535).astype(np.uint16)


def _expected(frames, dark, thresh, mult):
    n = len(frames)
    want = np.zeros((n, len(PATCHES), NP, NP), np.uint16)
    bgs = np.zeros(n, np.int64)
    for i in range(n):
        for b, (x, y) in enumerate(PATCHES):
            want[i, b], bgs[i] = oracle.preprocess_frame(frames[i], NP, (x, y), BK1, BK2, thresh, mult, bool(dark[i]))
    return want, bgs


def _solver(n):
    x0, y0, order = grid_geometry(NP, L, 3, 4)
    x0, y0 = x0[:n], y0[:n]
    order = np.arange(n)
    prob = fpm_amd.Problem(NP, L, order, x0, y0, R, 5, 10, n_patch=len(PATCHES))
    return fpm_amd.Solver(prob)


@pytest.mark.parametrize("thresh,mult", [(1000, 1.0), (2500, 3.0), (40000, 2.5)])
def test_frames_host_upload_matches_oracle(thresh, mult):
    n = 6
    frames = _frames(n)
    dark = np.array([1, 0, 1, 1, 0, 0], np.uint8)
    want, bgs = _expected(frames, dark, thresh, mult)
    with _solver(n) as s:
        bg = s.upload_frames(frames, [p[0] for p in PATCHES], [p[1] for p in PATCHES], BK1, BK2, thresh, mult, dark)
        got = s.download_stack()
    np.testing.assert_array_equal(bg, bgs)
    np.testing.assert_array_equal(got, want)


def test_frames_device_upload_and_solve():
    import torch
    n = 6
    frames = _frames(n, seed=4)
    dark = np.zeros(n, np.uint8)
    want, _ = _expected(frames, dark, 1000, 1.0)
    dev = torch.from_numpy(frames.view(np.int16)).cuda()
    with _solver(n) as s:
        s.upload_frames(None, [p[0] for p in PATCHES], [p[1] for p in PATCHES], BK1, BK2, 1000, 1.0, dark,
                        device_ptr=dev.data_ptr(), shape=(H, W))
        np.testing.assert_array_equal(s.download_stack(), want)
        s.init()
        s.run(1)
        out = s.download()
    # the same stack through the host upload gives the same reconstruction
    x0, y0, _ = grid_geometry(NP, L, 3, 4)
    prob = fpm_amd.Problem(NP, L, np.arange(n), x0[:n], y0[:n], R, 5, 10, n_patch=len(PATCHES))
    ref = fpm_amd.run_fpm(prob, want, 1)
    np.testing.assert_array_equal(out["objCrop"], ref["objCrop"])


def test_frames_reject_patch_outside():
    with _solver(6) as s:
        with pytest.raises(fpm_amd.FpmError, match="outside"):
            s.upload_frames(_frames(6), [0, 0, 0, W - NP + 1], [0, 0, 0, 0], BK1, BK2)
