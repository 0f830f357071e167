"""Np 90 fused kernel (csrc/fused_s90.hip: 90-point transforms in the
registers of 10-lane groups, dft90.hpp) -- the kernel BASELINE configs 1 and 2
(dataset_mono, Np 90) run on.  Checked against the C++ fp64 oracle and against
the generic small-patch kernel (FPM_NO_S90=1, fused_small.hip), which computes
the same step with Stockham passes: the two differ only by fp32 rounding of
different transform factorisations (bound in the assertion).

Tolerances as tests/test_gpu_parity.py: relative L2 of objF, objCrop and the
pupil <= 1e-5 after 1 iteration, <= 5e-5 after 2-3."""
import os

import numpy as np
import pytest

import fpm_amd
from fpm_oracle import rel_l2
from tools.synth import grid_geometry, make_stack

pytestmark = pytest.mark.gpu


def _solve(prob, stack, iters, generic=False):
    env = {"FPM_NO_S90": "1"} if generic else {}
    os.environ.update(env)
    try:
        with fpm_amd.Solver(prob) as s:
            want = fpm_amd.KERNEL_FUSED_SMALL if generic else fpm_amd.KERNEL_FUSED_NP90
            assert s.info().fused_kernel == want
            s.upload(stack)
            s.init()
            s.run(iters)
            return s.download()
    finally:
        for k in env:
            os.environ.pop(k, None)


CASES = [  # L, r, n_side, step, iters, B
    (360, 30, 4, 22, 2, 2),   # configs 1/2 optics on a synthetic grid
    (360, 12, 3, 30, 1, 1),
    (270, 44, 3, 20, 2, 2),   # the largest radius (2r + 1 = 89 box rows)
    (180, 3, 2, 10, 3, 3),
]


@pytest.mark.parametrize("L,r,nside,step,iters,B", CASES, ids=[f"r{c[1]}_it{c[4]}" for c in CASES])
def test_s90_matches_oracle_and_generic_small_kernel(L, r, nside, step, iters, B):
    import oracle_lib
    Np = 90
    x0, y0, order = grid_geometry(Np, L, nside, step)
    stack = make_stack(Np, L, r, x0, y0, n_patch=B, seed=91 + r)
    prob = fpm_amd.Problem(Np, L, order, x0, y0, r, 5, 10, n_patch=B, path=fpm_amd.PATH_FUSED)
    out = _solve(prob, stack, iters)
    # the generic kernel holds 4 box pixels per thread: (2r + 1)^2 <= 4096
    gen = _solve(prob, stack, iters, generic=True) if (2 * r + 1) ** 2 <= 4096 else None
    tol = 1e-5 if iters <= 1 else 5e-5
    for b in range(B):
        ref = oracle_lib.run_fpm(stack[:, b], order, x0, y0, Np, L, r, 5, 10, iters)
        for k in ("objF", "objCrop", "pupil"):
            e = rel_l2(out[k][b], ref[k])
            assert e < tol, (k, b, e)
            if gen is not None:
                eg = rel_l2(out[k][b], gen[k][b])
                assert eg < 2e-6, (k, b, eg)
    if B > 1:
        assert rel_l2(out["objCrop"][0], out["objCrop"][1]) > 1e-3  # patches differ


def test_s90_deterministic_and_iterations_compose():
    Np, L, r = 90, 360, 30
    x0, y0, order = grid_geometry(Np, L, 3, 30)
    stack = make_stack(Np, L, r, x0, y0, n_patch=2, seed=93)
    prob = fpm_amd.Problem(Np, L, order, x0, y0, r, 5, 10, n_patch=2, path=fpm_amd.PATH_FUSED)
    outs = []
    for split in (False, True):
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


def test_s90_lds_layouts_bit_identical():
    """The conflict-light LDS layout (r <= 30: shifted exchange tiles, T pitch
    106) and the dense one (FPM_S90_DENSE=1, also what r > 30 runs) move the
    same values through different LDS addresses: results are bit-identical."""
    Np, L, r = 90, 360, 30
    x0, y0, order = grid_geometry(Np, L, 4, 22)
    stack = make_stack(Np, L, r, x0, y0, n_patch=2, seed=95)
    prob = fpm_amd.Problem(Np, L, order, x0, y0, r, 5, 10, n_patch=2, path=fpm_amd.PATH_FUSED)
    fast = _solve(prob, stack, 2)
    os.environ["FPM_S90_DENSE"] = "1"
    try:
        dense = _solve(prob, stack, 2)
    finally:
        os.environ.pop("FPM_S90_DENSE", None)
    for k in ("objF", "objCrop", "pupil"):
        np.testing.assert_array_equal(fast[k], dense[k])
