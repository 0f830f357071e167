"""Np 256 register row/column kernels of the general path (csrc/np256.hip:
one 256-point transform per 16-lane group in registers, the stack read in the
fused column layout g = 16) for pupil radii beyond the fused Np 256 kernels
(r > 34; dataset_mono at cropSizeX 256 has r 84), vs the mixed-radix LDS
kernels they replace (FPM_NO_REG256=1 keeps the old ones) and vs the C++ fp64
oracle (GPU only).  The full-size dataset_mono case (64 patches, 193 LEDs)
is tests/test_gpu_configs.py::test_config2_geometry_at_np256_r84_64_patches.

Tolerance: relative L2 <= 1e-5 against the oracle after 1 iteration (as every
fp32 path), <= 1e-5 between the two GPU implementations after 2 iterations.
"""
import os

import numpy as np
import pytest

import fpm_amd
from fpm_oracle import rel_l2
from tools.synth import grid_geometry, make_stack

pytestmark = pytest.mark.gpu

Np = 256


def _run(prob, stack, iters, reg=True):
    if reg:
        os.environ.pop("FPM_NO_REG256", None)
    else:
        os.environ["FPM_NO_REG256"] = "1"
    try:
        return fpm_amd.run_fpm(prob, stack, iters)
    finally:
        os.environ.pop("FPM_NO_REG256", None)


@pytest.mark.parametrize("L,r,B", [(768, 84, 2), (768, 35, 3), (1024, 84, 8), (256, 127, 2)],
                         ids=["r84", "r35_3patches", "r84_8patches_xcd", "r127_edges"])
def test_np256_register_path_equals_lds_path(L, r, B):
    """B = 8 takes the XCD-aware block mapping (patch b on XCD b mod 8), the
    others the plain one; r 127 puts the support box at every frequency but
    the Nyquist row / column."""
    if L == Np:  # one LED: the crop covers the whole spectrum (crop 0, 0)
        x0, y0, order = np.array([0, 0]), np.array([0, 0]), [0, 1]
    else:
        x0, y0, order = grid_geometry(Np, L, 3 if L > 768 else 2, 60)
    stack = make_stack(Np, L, r, x0, y0, n_patch=B, seed=260 + r + B)
    prob = fpm_amd.Problem(Np, L, order, x0, y0, r, 5, 10, n_patch=B)
    with fpm_amd.Solver(prob) as s:
        assert s.info().path == fpm_amd.PATH_GENERAL
    reg = _run(prob, stack, 2, reg=True)
    lds = _run(prob, stack, 2, reg=False)
    for k in ("objF", "objCrop", "pupil"):
        for b in range(B):
            e = rel_l2(reg[k][b], lds[k][b])
            assert e < 1e-5, (k, b, e)


def test_np256_register_path_vs_oracle():
    import oracle_lib
    L, r = 768, 84
    x0, y0, order = grid_geometry(Np, L, 3, 50)
    stack = make_stack(Np, L, r, x0, y0, n_patch=1, seed=265)
    prob = fpm_amd.Problem(Np, L, order, x0, y0, r, 5, 10, n_patch=1)
    out = _run(prob, stack, 1)
    ref = oracle_lib.run_fpm(stack[:, 0], order, x0, y0, Np, L, r, 5, 10, 1)
    for k in ("objF", "objCrop", "pupil"):
        e = rel_l2(out[k][0], ref[k])
        print(f"np256 register path r 84 {k} rel L2 {e:.2e}")
        assert e < 1e-5, k


def test_np256_register_path_stack_layout_round_trip():
    L, r = 768, 84
    x0, y0, order = grid_geometry(Np, L, 2, 60)
    rng = np.random.default_rng(266)
    stack = rng.integers(0, 65535, (len(x0), 2, Np, Np)).astype(np.uint16)
    with fpm_amd.Solver(fpm_amd.Problem(Np, L, order, x0, y0, r, 5, 10, n_patch=2)) as s:
        s.upload(stack)
        np.testing.assert_array_equal(s.download_stack(), stack)
