"""HIP path vs the CPU oracle on seeded synthetic stacks (GPU only).

Tolerance (stated here, DESIGN.md "Parity"): the HIP path keeps complex
float32 state against the oracle's complex128; relative L2 error of objCrop,
objF and the pupil must stay below 1e-5 after 1 iteration and 5e-5 after 3.
Measured drift of an fp32 restatement of the same algorithm is ~1e-7 to 4e-7
(5 iterations, Np 32/64), so this bound has >20x margin and would still catch
any indexing, sign, scaling or ordering error (those give O(1) errors).
"""
import numpy as np
import pytest

from fpm_oracle import run_fpm as oracle_run, rel_l2
import fpm_amd
from tools.synth import make_stack, grid_geometry

pytestmark = pytest.mark.gpu

CASES = [
    # Np, L, r, n_side, step, iters, delta1, delta2, path
    (32, 96, 6, 5, 4, 1, 5, 10, fpm_amd.PATH_GENERAL),
    (32, 96, 6, 5, 4, 3, 5, 10, fpm_amd.PATH_GENERAL),
    (64, 192, 10, 7, 6, 2, 10, 3, fpm_amd.PATH_GENERAL),
    (30, 90, 5, 5, 4, 2, 5, 10, fpm_amd.PATH_GENERAL),      # radix 2*3*5
    (40, 120, 7, 3, 9, 2, 1000, 70, fpm_amd.PATH_GENERAL),  # radix 2^3*5, 3*2^3*5
]


def _tol(iters):
    return 1e-5 if iters <= 1 else 5e-5


@pytest.mark.parametrize("case", CASES, ids=lambda c: f"Np{c[0]}_L{c[1]}_r{c[2]}_it{c[5]}")
def test_single_patch_matches_oracle(case):
    Np, L, r, nside, step, iters, d1, d2, path = case
    x0, y0, order = grid_geometry(Np, L, nside, step)
    stack = make_stack(Np, L, r, x0, y0, n_patch=1)
    ref = oracle_run(stack[:, 0], order, x0, y0, Np, L, r, d1, d2, iters)
    prob = fpm_amd.Problem(Np, L, order, x0, y0, r, d1, d2, n_patch=1, path=path)
    out = fpm_amd.run_fpm(prob, stack, iters)
    tol = _tol(iters)
    assert rel_l2(out["objF"][0], ref["objF"]) < tol
    assert rel_l2(out["objCrop"][0], ref["objCrop"]) < tol
    assert rel_l2(out["pupil"][0], ref["pupil"]) < tol
    np.testing.assert_array_equal(out["support"][0], ref["support"].real.astype(np.float32))


def test_batched_patches_are_independent():
    """B patches in one context == each patch run alone through the oracle."""
    Np, L, r, iters = 32, 96, 6, 2
    x0, y0, order = grid_geometry(Np, L, 5, 4)
    B = 3
    stack = make_stack(Np, L, r, x0, y0, n_patch=B, seed=7)
    prob = fpm_amd.Problem(Np, L, order, x0, y0, r, 5, 10, n_patch=B, path=fpm_amd.PATH_GENERAL)
    out = fpm_amd.run_fpm(prob, stack, iters)
    for b in range(B):
        ref = oracle_run(stack[:, b], order, x0, y0, Np, L, r, 5, 10, iters)
        assert rel_l2(out["objCrop"][b], ref["objCrop"]) < _tol(iters)
        assert rel_l2(out["pupil"][b], ref["pupil"]) < _tol(iters)


@pytest.mark.parametrize("all_channels", [True, False], ids=["opencv_scalar", "re_only"])
def test_metric_geometry_patch_vs_cpp_oracle(all_channels):
    """Full metric size (dogStomach optics, 293 LEDs, Np 256, L 768, r 33),
    one iteration, against the C++ fp64 oracle run on the same box, for both
    readings of cv::add(UMat c2, double)."""
    import bench
    import oracle_lib
    geo = bench.metric_geometry()
    order = np.arange(geo["n_led"])
    stack = make_stack(geo["np_"], geo["L"], geo["r"], geo["x0"], geo["y0"], n_patch=1, seed=5)
    ref = oracle_lib.run_fpm(stack[:, 0], order, geo["x0"], geo["y0"], geo["np_"], geo["L"], geo["r"],
                             geo["d1"], geo["d2"], 1, all_channels=all_channels)
    flags = 0 if all_channels else fpm_amd.FLAG_SCALAR_RE_ONLY
    for path in (fpm_amd.PATH_GENERAL, fpm_amd.PATH_AUTO):
        prob = fpm_amd.Problem(geo["np_"], geo["L"], order, geo["x0"], geo["y0"], geo["r"], geo["d1"],
                               geo["d2"], n_patch=1, path=path, flags=flags)
        out = fpm_amd.run_fpm(prob, stack, 1)
        assert rel_l2(out["objCrop"][0], ref["objCrop"]) < 1e-5
        assert rel_l2(out["objF"][0], ref["objF"]) < 1e-5
        assert rel_l2(out["pupil"][0], ref["pupil"]) < 1e-5


def test_golden_fixtures_on_gpu():
    import glob
    import os
    for path in sorted(glob.glob(os.path.join(os.path.dirname(__file__), "golden", "solver_*.npz"))):
        g = np.load(path)
        Np, L, r, iters, d1, d2 = (int(v) for v in g["params"])
        flags = 0 if int(g["all_channels"]) else fpm_amd.FLAG_SCALAR_RE_ONLY
        prob = fpm_amd.Problem(Np, L, g["order"], g["x0"], g["y0"], r, d1, d2, flags=flags)
        out = fpm_amd.run_fpm(prob, g["stack"], iters)
        for k in ("objF", "objCrop", "pupil"):
            assert rel_l2(out[k][0], g[k]) < _tol(iters), (path, k)


FUSED_CASES = [
    # r, n_side, step, iters: NB = 2r+1 rows; > 64 rows exercises the tail-row direct DFTs
    (10, 5, 24, 2),
    (31, 3, 40, 2),     # NB 63: every row on the FFT groups
    (32, 3, 40, 2),     # NB 65: one tail row
    (33, 5, 20, 2),     # NB 67: the metric radius, three tail rows
    (34, 3, 30, 3),     # NB 69: five tail rows, 59 tail pixels
]


@pytest.mark.parametrize("case", FUSED_CASES, ids=lambda c: f"r{c[0]}_leds{c[1]**2}_it{c[3]}")
def test_fused_path_matches_oracle(case):
    r, nside, step, iters = case
    Np, L = 256, 512
    x0, y0, order = grid_geometry(Np, L, nside, step)
    stack = make_stack(Np, L, r, x0, y0, n_patch=2, seed=21)
    prob = fpm_amd.Problem(Np, L, order, x0, y0, r, 10, 3, n_patch=2, path=fpm_amd.PATH_FUSED)
    with fpm_amd.Solver(prob) as s:
        assert s.info().path == fpm_amd.PATH_FUSED
        s.upload(stack)
        s.init()
        s.run(iters)
        out = s.download()
    import oracle_lib
    for b in range(2):
        ref = oracle_lib.run_fpm(stack[:, b], order, x0, y0, Np, L, r, 10, 3, iters)
        assert rel_l2(out["objF"][b], ref["objF"]) < _tol(iters)
        assert rel_l2(out["objCrop"][b], ref["objCrop"]) < _tol(iters)
        assert rel_l2(out["pupil"][b], ref["pupil"]) < _tol(iters)


def test_fused_equals_general_path():
    """Both device paths on the same inputs agree to fp32 rounding."""
    Np, L, r, iters = 256, 512, 33, 2
    x0, y0, order = grid_geometry(Np, L, 5, 20)
    stack = make_stack(Np, L, r, x0, y0, n_patch=1, seed=22)
    outs = {}
    for path in (fpm_amd.PATH_GENERAL, fpm_amd.PATH_FUSED):
        prob = fpm_amd.Problem(Np, L, order, x0, y0, r, 10, 3, path=path)
        outs[path] = fpm_amd.run_fpm(prob, stack, iters)
    for k in ("objF", "objCrop", "pupil"):
        assert rel_l2(outs[fpm_amd.PATH_FUSED][k], outs[fpm_amd.PATH_GENERAL][k]) < 2e-6


def test_unsupported_fused_radius_falls_back_to_general():
    Np, L, r = 256, 512, 40
    x0, y0, order = grid_geometry(Np, L, 3, 30)
    prob = fpm_amd.Problem(Np, L, order, x0, y0, r, 10, 3, path=fpm_amd.PATH_AUTO)
    with fpm_amd.Solver(prob) as s:
        assert s.info().path == fpm_amd.PATH_GENERAL
    with pytest.raises(fpm_amd.FpmError):
        fpm_amd.Solver(fpm_amd.Problem(Np, L, order, x0, y0, r, 10, 3, path=fpm_amd.PATH_FUSED))


@pytest.mark.parametrize("path", [fpm_amd.PATH_GENERAL, fpm_amd.PATH_FUSED])
def test_iterations_compose_and_runs_are_deterministic(path):
    """run(2) == run(1); run(1) bit for bit (the state carried between launches
    -- spectrum, pupil, tile maxima, dirty bits, max|P| -- is complete), and two
    contexts on the same input give identical bits (no order-dependent atomics)."""
    Np, L, r = 256, 512, 33
    x0, y0, order = grid_geometry(Np, L, 3, 24)
    stack = make_stack(Np, L, r, x0, y0, n_patch=2, seed=31)
    prob = fpm_amd.Problem(Np, L, order, x0, y0, r, 10, 3, n_patch=2, path=path)
    outs = []
    for split in (False, True, True):
        with fpm_amd.Solver(prob) as s:
            s.upload(stack)
            s.init()
            if split:
                s.run(1)
                s.run(1)
            else:
                s.run(2)
            outs.append(s.download())
    for k in ("objF", "objCrop", "pupil"):
        np.testing.assert_array_equal(outs[0][k], outs[1][k])
        np.testing.assert_array_equal(outs[1][k], outs[2][k])


def test_objcrop_last_only_flag():
    Np, L, r = 256, 768, 33
    x0, y0, order = grid_geometry(Np, L, 3, 24)
    stack = make_stack(Np, L, r, x0, y0, n_patch=1, seed=32)
    a = fpm_amd.run_fpm(fpm_amd.Problem(Np, L, order, x0, y0, r, 10, 3), stack, 2)
    b = fpm_amd.run_fpm(fpm_amd.Problem(Np, L, order, x0, y0, r, 10, 3, flags=fpm_amd.FLAG_OBJCROP_LAST_ONLY),
                        stack, 2)
    for k in ("objF", "objCrop", "pupil"):
        np.testing.assert_array_equal(a[k], b[k])


def test_fused_more_patches_than_cus():
    """n_patch > 256: the fused grid runs in more than one wave of workgroups."""
    import oracle_lib
    Np, L, r, B = 256, 512, 33, 260
    x0, y0, order = grid_geometry(Np, L, 2, 24)
    rng = np.random.default_rng(33)
    stack = rng.integers(0, 30000, (len(x0), B, Np, Np)).astype(np.uint16)
    prob = fpm_amd.Problem(Np, L, order, x0, y0, r, 10, 3, n_patch=B, path=fpm_amd.PATH_FUSED)
    out = fpm_amd.run_fpm(prob, stack, 1)
    for b in (0, 255, 259):
        ref = oracle_lib.run_fpm(stack[:, b], order, x0, y0, Np, L, r, 10, 3, 1)
        assert rel_l2(out["objCrop"][b], ref["objCrop"]) < 1e-5
        assert rel_l2(out["pupil"][b], ref["pupil"]) < 1e-5


@pytest.mark.parametrize("Np,L,r", [(200, 600, 26), (90, 360, 30), (64, 192, 10)])
def test_wave_and_tiled_column_passes_agree(Np, L, r, monkeypatch):
    """The wave-private column pass (k_colpass_wave, the default wherever a
    wave holds >= 2 columns) and the block-tiled one (k_colpass_tiled,
    FPM_NO_WAVE_COLS=1) compute the same transforms with different pass
    orders: both match the oracle and each other far inside the tolerance."""
    x0, y0, order = grid_geometry(Np, L, 3, max(1, r // 3))
    stack = make_stack(Np, L, r, x0, y0, n_patch=2, seed=11)
    prob = fpm_amd.Problem(Np, L, order, x0, y0, r, 5, 10, n_patch=2, path=fpm_amd.PATH_GENERAL)
    wave = fpm_amd.run_fpm(prob, stack, 2)
    monkeypatch.setenv("FPM_NO_WAVE_COLS", "1")
    tiled = fpm_amd.run_fpm(prob, stack, 2)
    ref = oracle_run(stack[:, 1], order, x0, y0, Np, L, r, 5, 10, 2)
    for out in (wave, tiled):
        assert rel_l2(out["objCrop"][1], ref["objCrop"]) < _tol(2)
        assert rel_l2(out["pupil"][1], ref["pupil"]) < _tol(2)
    for b in range(2):
        assert rel_l2(wave["objCrop"][b], tiled["objCrop"][b]) < 2e-6
        assert rel_l2(wave["pupil"][b], tiled["pupil"][b]) < 2e-6


@pytest.mark.parametrize("Np,L,step", [(256, 512, 60), (256, 768, 100), (256, 1024, 150), (200, 600, 80),
                                       (90, 360, 40)])
def test_objcrop_live_band(Np, L, step):
    """objCrop transforms only the live band of the spectrum (rows/columns the
    init placement and the used LEDs' support boxes reach, fpm_state.hpp):
    with an LED set off to one side the band is asymmetric, the spectrum is
    exactly zero outside it, and objCrop still equals the dense IDFT of objF
    (numpy, complex128) computed from the GPU's own spectrum."""
    # L 600 / 360: the Np 200 / Np 90 kernels and the 600- / 360-point objCrop passes
    r = {256: 33, 200: 26, 90: 30}[Np]
    c = L // 2 - Np // 2
    x0 = np.array([c, c + step, c + 2 * step, c + step])
    y0 = np.array([c, c, c - step, c - 2 * step])
    order = [0, 1, 2, 3]
    stack = make_stack(Np, L, r, x0, y0, n_patch=1, seed=41)
    out = fpm_amd.run_fpm(fpm_amd.Problem(Np, L, order, x0, y0, r, 10, 3), stack, 1)
    spec = np.fft.fftshift(out["objF"][0])
    sy0, sy1 = min(L // 2 - r, y0.min() + Np // 2 - r), max(L // 2 + r, y0.max() + Np // 2 + r)
    sx0, sx1 = min(L // 2 - r, x0.min() + Np // 2 - r), max(L // 2 + r, x0.max() + Np // 2 + r)
    assert sy1 - sy0 + 1 < L and sx1 - sx0 + 1 < L
    live = np.zeros((L, L), bool)
    live[sy0:sy1 + 1, sx0:sx1 + 1] = True
    assert np.count_nonzero(spec[~live]) == 0
    assert np.count_nonzero(spec[live]) > 0
    ref = np.fft.ifft2(out["objF"][0].astype(np.complex128))
    assert rel_l2(out["objCrop"][0], ref) < 2e-6
