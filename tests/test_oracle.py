"""The CPU oracles (numpy oracle/fpm_oracle.py, C++ oracle/liboracle.so)
against known answers and the committed golden vectors.  CPU only.

The reference ships no fixtures and cannot be built here, so
the cvComplex semantics are pinned by these known-answer tests:
  (i)   fft2 = unscaled DFT, ifft2 = DFT^-1 scaled 1/N   -> FFT KAT vs numpy
  (iii) fftShift = quadrant swap (even sizes)             -> shift KAT
  (v)   filled cv::circle == Euclidean disk               -> support pixel
        counts the survey measured on an emulation of OpenCV's fill
        (r = 26/30/33/84 -> 2121/2821/3409/22133)
and the two independent restatements (numpy, C++) must agree to ~1e-12.
"""
import glob
import os

import numpy as np
import pytest

import oracle_lib
from fpm_oracle import disk_support, fftshift2, rel_l2, run_fpm

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


@pytest.mark.parametrize("shape", [(32, 32), (30, 90), (200, 40), (96, 96), (768, 4), (10, 750)])
def test_cpp_fft_matches_numpy(shape):
    rng = np.random.default_rng(1)
    a = rng.standard_normal(shape) + 1j * rng.standard_normal(shape)
    np.testing.assert_allclose(oracle_lib.fft2(a), np.fft.fft2(a), rtol=0, atol=1e-9 * np.abs(a).sum() / a.size**0.5)
    np.testing.assert_allclose(oracle_lib.fft2(a, inverse=True), np.fft.ifft2(a), rtol=0, atol=1e-12 * np.abs(a).sum())


def test_fftshift_is_quadrant_swap():
    a = np.arange(36).reshape(6, 6)
    s = fftshift2(a)
    assert s[3, 3] == a[0, 0] and s[0, 0] == a[3, 3] and s[0, 3] == a[3, 0]
    np.testing.assert_array_equal(fftshift2(s), a)


@pytest.mark.parametrize("r,count", [(26, 2121), (30, 2821), (33, 3409), (84, 22133)])
def test_support_disk_pixel_counts(r, count):
    np_ = 2 * r + 40
    s = disk_support(np_, r)
    assert int(s.sum()) == count
    assert s[0, 0] == 1  # un-centred: DC at [0, 0]


@pytest.mark.parametrize("path", sorted(glob.glob(os.path.join(GOLDEN, "solver_*.npz"))),
                         ids=lambda p: os.path.basename(p)[7:-4])
def test_oracles_reproduce_golden(path):
    g = np.load(path)
    Np, L, r, iters, d1, d2 = (int(v) for v in g["params"])
    py = run_fpm(g["stack"], g["order"], g["x0"], g["y0"], Np, L, r, d1, d2, iters)
    cc = oracle_lib.run_fpm(g["stack"], g["order"], g["x0"], g["y0"], Np, L, r, d1, d2, iters)
    for k in ("objF", "objCrop", "pupil"):
        assert rel_l2(py[k], g[k]) < 1e-6, k      # fixture stored as complex64
        assert rel_l2(cc[k], py[k]) < 1e-10, k    # two fp64 restatements agree


def test_cpp_batch_equals_single():
    g = np.load(os.path.join(GOLDEN, "solver_np32_r6_it2.npz"))
    Np, L, r, iters, d1, d2 = (int(v) for v in g["params"])
    st = np.stack([g["stack"], g["stack"][::-1, ::-1, :]], axis=1)   # two different patches
    batch = oracle_lib.run_fpm_batch(st, g["order"], g["x0"], g["y0"], Np, L, r, d1, d2, iters, threads=2)
    for b in range(2):
        one = oracle_lib.run_fpm(st[:, b], g["order"], g["x0"], g["y0"], Np, L, r, d1, d2, iters)
        assert rel_l2(batch[b], one["objCrop"]) == 0.0
