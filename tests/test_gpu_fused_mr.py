"""Np 200 fused kernel (csrc/fused_mr.hip: 20 x 10 register four-step, one
768-thread workgroup per patch) vs the C++ fp64 oracle and vs the general
path (GPU only).  BASELINE config 3 (dataset_dogStomach.json literal: Np 200,
L 600, naRadius 26, 157 LEDs, 256 patches) runs on this kernel; its literal
geometry test is tests/test_gpu_configs.py::test_config3_dogstomach_literal_256_patches.

Tolerance as in tests/test_gpu_parity.py: relative L2 of objF, objCrop and the
pupil <= 1e-5 after 1 iteration, <= 5e-5 after 2-3; fused vs general < 2e-6.
"""
import numpy as np
import pytest

import fpm_amd
from fpm_oracle import rel_l2
from tools.synth import grid_geometry, make_stack

pytestmark = pytest.mark.gpu

Np, L = 200, 600


def _tol(iters):
    return 1e-5 if iters <= 1 else 5e-5


@pytest.mark.parametrize("r,nside,step,iters", [(26, 3, 30, 2), (10, 4, 12, 2), (29, 3, 25, 3), (1, 2, 3, 1)],
                         ids=["r26", "r10", "r29_max", "r1"])
def test_np200_fused_matches_oracle(r, nside, step, iters):
    import oracle_lib
    x0, y0, order = grid_geometry(Np, L, nside, step)
    stack = make_stack(Np, L, r, x0, y0, n_patch=2, seed=61 + r)
    prob = fpm_amd.Problem(Np, L, order, x0, y0, r, 10, 3, n_patch=2, path=fpm_amd.PATH_FUSED)
    with fpm_amd.Solver(prob) as s:
        assert s.info().path == fpm_amd.PATH_FUSED
        s.upload(stack)
        s.init()
        s.run(iters)
        out = s.download()
    for b in range(2):
        ref = oracle_lib.run_fpm(stack[:, b], order, x0, y0, Np, L, r, 10, 3, iters)
        for k in ("objF", "objCrop", "pupil"):
            e = rel_l2(out[k][b], ref[k])
            assert e < _tol(iters), (k, b, e)


def test_np200_fused_equals_general_path():
    r, iters = 26, 2
    x0, y0, order = grid_geometry(Np, L, 4, 20)
    stack = make_stack(Np, L, r, x0, y0, n_patch=2, seed=65)
    outs = {}
    for path in (fpm_amd.PATH_GENERAL, fpm_amd.PATH_FUSED):
        prob = fpm_amd.Problem(Np, L, order, x0, y0, r, 10, 3, n_patch=2, path=path)
        outs[path] = fpm_amd.run_fpm(prob, stack, iters)
    for k in ("objF", "objCrop", "pupil"):
        for b in range(2):
            assert rel_l2(outs[fpm_amd.PATH_FUSED][k][b], outs[fpm_amd.PATH_GENERAL][k][b]) < 2e-6, (k, b)


def test_np200_iterations_compose_and_are_deterministic():
    r = 26
    x0, y0, order = grid_geometry(Np, L, 3, 30)
    stack = make_stack(Np, L, r, x0, y0, n_patch=2, seed=66)
    prob = fpm_amd.Problem(Np, L, order, x0, y0, r, 10, 3, n_patch=2, path=fpm_amd.PATH_FUSED)
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


def test_np200_radius_beyond_slots_falls_back_to_general():
    r = 30  # the six slot registers cover |k| <= 29
    x0, y0, order = grid_geometry(Np, L, 3, 30)
    with fpm_amd.Solver(fpm_amd.Problem(Np, L, order, x0, y0, r, 10, 3)) as s:
        assert s.info().path == fpm_amd.PATH_GENERAL
    with pytest.raises(fpm_amd.FpmError):
        fpm_amd.Solver(fpm_amd.Problem(Np, L, order, x0, y0, r, 10, 3, path=fpm_amd.PATH_FUSED))


def test_np200_more_patches_than_cus():
    import oracle_lib
    r, B = 26, 258
    x0, y0, order = grid_geometry(Np, L, 2, 30)
    rng = np.random.default_rng(67)
    stack = rng.integers(0, 30000, (len(x0), B, Np, Np)).astype(np.uint16)
    prob = fpm_amd.Problem(Np, L, order, x0, y0, r, 10, 3, n_patch=B, path=fpm_amd.PATH_FUSED)
    out = fpm_amd.run_fpm(prob, stack, 1)
    for b in (0, 129, 257):
        ref = oracle_lib.run_fpm(stack[:, b], order, x0, y0, Np, L, r, 10, 3, 1)
        assert rel_l2(out["objCrop"][b], ref["objCrop"]) < 1e-5, b
        assert rel_l2(out["pupil"][b], ref["pupil"]) < 1e-5, b


def test_np200_lds_layouts_bit_identical():
    """Bank-friendly strides (exchange-tile stride 106, T pitch 202, whatever
    LDS allows) and the dense layout (FPM_MR_DENSE=1) move the same values
    through different LDS addresses: bit-identical results."""
    import os
    r, iters = 26, 2
    x0, y0, order = grid_geometry(Np, L, 4, 20)
    stack = make_stack(Np, L, r, x0, y0, n_patch=2, seed=67)
    prob = fpm_amd.Problem(Np, L, order, x0, y0, r, 10, 3, n_patch=2, path=fpm_amd.PATH_FUSED)
    outs = []
    for dense in (False, True):
        if dense:
            os.environ["FPM_MR_DENSE"] = "1"
        try:
            outs.append(fpm_amd.run_fpm(prob, stack, iters))
        finally:
            os.environ.pop("FPM_MR_DENSE", None)
    for k in ("objF", "objCrop", "pupil"):
        np.testing.assert_array_equal(outs[0][k], outs[1][k])
