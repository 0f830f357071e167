"""Small-patch fused kernel (csrc/fused_small.hip: one 1024-thread workgroup
per patch, the sub-aperture field in LDS, mixed-radix Stockham passes) vs the
C++ fp64 oracle and vs the general path (GPU only).  BASELINE configs 1 and 2
(dataset_mono geometry: Np 90, L 360, naRadius 30) run on this kernel; their
literal-geometry tests are in tests/test_gpu_configs.py.

Tolerance as in tests/test_gpu_parity.py: relative L2 of objF, objCrop and the
pupil <= 1e-5 after 1 iteration, <= 5e-5 after 2-3; fused vs general < 2e-6.
"""
import numpy as np
import pytest

import fpm_amd
from fpm_oracle import rel_l2
from tools.synth import grid_geometry, make_stack

pytestmark = pytest.mark.gpu


def _tol(iters):
    return 1e-5 if iters <= 1 else 5e-5


CASES = [  # Np, L, r, n_side, step, iters
    (90, 360, 30, 4, 22, 2),   # configs 1/2 optics on a synthetic grid
    (90, 360, 12, 3, 30, 1),
    (64, 192, 20, 3, 16, 2),   # radix 8 x 8
    (96, 288, 31, 3, 24, 3),   # the largest Np and r the kernel takes
    (30, 90, 6, 5, 9, 2),      # 2 x 3 x 5
    (8, 24, 1, 2, 3, 1),
]


@pytest.mark.parametrize("Np,L,r,nside,step,iters", CASES,
                         ids=[f"np{c[0]}_r{c[2]}" for c in CASES])
def test_small_fused_matches_oracle(Np, L, r, nside, step, iters):
    import oracle_lib
    x0, y0, order = grid_geometry(Np, L, nside, step)
    stack = make_stack(Np, L, r, x0, y0, n_patch=2, seed=71 + Np + r)
    prob = fpm_amd.Problem(Np, L, order, x0, y0, r, 5, 10, n_patch=2, path=fpm_amd.PATH_FUSED)
    with fpm_amd.Solver(prob) as s:
        assert s.info().path == fpm_amd.PATH_FUSED
        s.upload(stack)
        s.init()
        s.run(iters)
        out = s.download()
    for b in range(2):
        ref = oracle_lib.run_fpm(stack[:, b], order, x0, y0, Np, L, r, 5, 10, iters)
        for k in ("objF", "objCrop", "pupil"):
            e = rel_l2(out[k][b], ref[k])
            assert e < _tol(iters), (k, b, e)


def test_small_fused_re_only_semantics():
    import oracle_lib
    Np, L, r = 90, 360, 30
    x0, y0, order = grid_geometry(Np, L, 3, 25)
    stack = make_stack(Np, L, r, x0, y0, n_patch=1, seed=78)
    prob = fpm_amd.Problem(Np, L, order, x0, y0, r, 5, 10, n_patch=1, path=fpm_amd.PATH_FUSED,
                           flags=fpm_amd.FLAG_SCALAR_RE_ONLY)
    out = fpm_amd.run_fpm(prob, stack, 2)
    ref = oracle_lib.run_fpm(stack[:, 0], order, x0, y0, Np, L, r, 5, 10, 2, all_channels=False)
    for k in ("objF", "objCrop", "pupil"):
        assert rel_l2(out[k][0], ref[k]) < 5e-5, k


def test_small_fused_equals_general_path():
    Np, L, r, iters = 90, 360, 30, 2
    x0, y0, order = grid_geometry(Np, L, 5, 18)
    stack = make_stack(Np, L, r, x0, y0, n_patch=3, seed=72)
    outs = {}
    for path in (fpm_amd.PATH_GENERAL, fpm_amd.PATH_FUSED):
        prob = fpm_amd.Problem(Np, L, order, x0, y0, r, 5, 10, n_patch=3, path=path)
        outs[path] = fpm_amd.run_fpm(prob, stack, iters)
    for k in ("objF", "objCrop", "pupil"):
        for b in range(3):
            assert rel_l2(outs[fpm_amd.PATH_FUSED][k][b], outs[fpm_amd.PATH_GENERAL][k][b]) < 2e-6, (k, b)


def test_small_iterations_compose_and_are_deterministic():
    Np, L, r = 90, 360, 30
    x0, y0, order = grid_geometry(Np, L, 3, 30)
    stack = make_stack(Np, L, r, x0, y0, n_patch=2, seed=73)
    prob = fpm_amd.Problem(Np, L, order, x0, y0, r, 5, 10, n_patch=2, path=fpm_amd.PATH_FUSED)
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


def test_small_stack_layout_round_trip():
    """The fused kernel reads the stack transposed in place; the download hands
    back the C-ABI layout bit for bit."""
    Np, L, r = 90, 360, 30
    x0, y0, order = grid_geometry(Np, L, 2, 30)
    rng = np.random.default_rng(74)
    stack = rng.integers(0, 65535, (len(x0), 3, Np, Np)).astype(np.uint16)
    with fpm_amd.Solver(fpm_amd.Problem(Np, L, order, x0, y0, r, 5, 10, n_patch=3)) as s:
        assert s.info().path == fpm_amd.PATH_FUSED
        s.upload(stack)
        np.testing.assert_array_equal(s.download_stack(), stack)


def test_small_radius_beyond_registers_falls_back_to_general():
    Np, L, r = 96, 288, 32  # (2r+1)^2 = 4225 > 1024 threads x 4 pixels
    x0, y0, order = grid_geometry(Np, L, 2, 30)
    with fpm_amd.Solver(fpm_amd.Problem(Np, L, order, x0, y0, r, 5, 10)) as s:
        assert s.info().path == fpm_amd.PATH_GENERAL
    with pytest.raises(fpm_amd.FpmError):
        fpm_amd.Solver(fpm_amd.Problem(Np, L, order, x0, y0, r, 5, 10, path=fpm_amd.PATH_FUSED))


def test_small_more_patches_than_cus():
    import oracle_lib
    Np, L, r, B = 90, 360, 30, 260
    x0, y0, order = grid_geometry(Np, L, 2, 20)
    rng = np.random.default_rng(75)
    stack = rng.integers(0, 30000, (len(x0), B, Np, Np)).astype(np.uint16)
    prob = fpm_amd.Problem(Np, L, order, x0, y0, r, 5, 10, n_patch=B, path=fpm_amd.PATH_FUSED)
    out = fpm_amd.run_fpm(prob, stack, 1)
    for b in (0, 131, 259):
        ref = oracle_lib.run_fpm(stack[:, b], order, x0, y0, Np, L, r, 5, 10, 1)
        assert rel_l2(out["objCrop"][b], ref["objCrop"]) < 1e-5, b
        assert rel_l2(out["pupil"][b], ref["pupil"]) < 1e-5, b
