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
(iv) is OpenCV's published scalar rule (cv::add / cv::multiply of a CV_64FC2
array and a double act on every channel); test_scalar_semantics_differ shows
the two readings give measurably different reconstructions.
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
    allc = bool(g["all_channels"])
    py = run_fpm(g["stack"], g["order"], g["x0"], g["y0"], Np, L, r, d1, d2, iters, all_channels=allc)
    cc = oracle_lib.run_fpm(g["stack"], g["order"], g["x0"], g["y0"], Np, L, r, d1, d2, iters, all_channels=allc)
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


def test_scalar_semantics_differ():
    """The complex denominators of fpmMain.cpp:417-419/469-471 (OpenCV scalar
    unrolling) are not a rounding-level change: after one iteration the two
    readings differ by far more than any parity tolerance."""
    g = np.load(os.path.join(GOLDEN, "solver_np32_r6_it2.npz"))
    Np, L, r, iters, d1, d2 = (int(v) for v in g["params"])
    a = oracle_lib.run_fpm(g["stack"], g["order"], g["x0"], g["y0"], Np, L, r, d1, d2, 1, all_channels=True)
    b = oracle_lib.run_fpm(g["stack"], g["order"], g["x0"], g["y0"], Np, L, r, d1, d2, 1, all_channels=False)
    assert rel_l2(a["objCrop"], b["objCrop"]) > 1e-3
    assert rel_l2(a["pupil"], b["pupil"]) > 1e-3


def test_complex_denominator_restatement():
    """One LED step of the numpy oracle against a hand-written complex division
    (num / ((|P|^2 + d2 + i d2) max|P|)): checks the unrolled-scalar reading
    op by op on random data."""
    rng = np.random.default_rng(3)
    P = rng.standard_normal((8, 8)) + 1j * rng.standard_normal((8, 8))
    num = rng.standard_normal((8, 8)) + 1j * rng.standard_normal((8, 8))
    d2 = 3.0
    pa = np.abs(P)
    den = (pa * pa + d2 + 1j * d2) * pa.max()
    want = num * (pa * pa + d2 - 1j * d2) / (((pa * pa + d2) ** 2 + d2 * d2) * pa.max())
    np.testing.assert_allclose(num / den, want, rtol=1e-13)
