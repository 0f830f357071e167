"""Np 1024 register row/column kernels of the general path (csrc/np1024.hip:
1024-point transforms in the registers of 16-lane groups, the stack read
transposed) vs the mixed-radix LDS kernels they replace (FPM_NO_REG1024=1
keeps the old ones) and vs the C++ fp64 oracle (GPU only).  BASELINE config 5
(Np 1024, L 4096, naRadius 333, fp16 storage) runs on them; its full-size tests
are tests/test_gpu_configs.py::test_config5_*.

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

Np = 1024


def _run(prob, stack, iters, reg=True):
    if reg:
        os.environ.pop("FPM_NO_REG1024", None)
    else:
        os.environ["FPM_NO_REG1024"] = "1"
    try:
        return fpm_amd.run_fpm(prob, stack, iters)
    finally:
        os.environ.pop("FPM_NO_REG1024", None)


@pytest.mark.parametrize("L,r,fp16", [(2048, 333, False), (2048, 120, False), (2048, 333, True), (1024, 511, False)],
                         ids=["r333", "r120", "r333_fp16", "r511_edges"])
def test_np1024_register_path_equals_lds_path(L, r, fp16):
    if L == Np:  # one LED: the crop covers the whole spectrum (crop 0, 0)
        x0, y0, order = np.array([0, 0]), np.array([0, 0]), [0, 1]
    else:
        x0, y0, order = grid_geometry(Np, L, 2, 100)
    stack = make_stack(Np, L, r, x0, y0, n_patch=2, seed=81 + r)
    flags = fpm_amd.FLAG_SPEC_FP16 if fp16 else 0
    prob = fpm_amd.Problem(Np, L, order, x0, y0, r, 5, 10, n_patch=2, flags=flags)
    reg = _run(prob, stack, 2, reg=True)
    lds = _run(prob, stack, 2, reg=False)
    tol = 2e-3 if fp16 else 1e-5  # fp16: the two paths round different fp32 values on each store
    for k in ("objF", "objCrop", "pupil"):
        for b in range(2):
            assert rel_l2(reg[k][b], lds[k][b]) < tol, (k, b)


def test_np1024_register_path_vs_oracle():
    import oracle_lib
    L, r = 2048, 333
    x0, y0, order = grid_geometry(Np, L, 2, 150)
    stack = make_stack(Np, L, r, x0, y0, n_patch=1, seed=85)
    prob = fpm_amd.Problem(Np, L, order, x0, y0, r, 5, 10, n_patch=1)
    out = _run(prob, stack, 1)
    ref = oracle_lib.run_fpm(stack[:, 0], order, x0, y0, Np, L, r, 5, 10, 1)
    for k in ("objF", "objCrop", "pupil"):
        assert rel_l2(out[k][0], ref[k]) < 1e-5, k


def test_np1024_stack_layout_round_trip():
    L, r = 2048, 333
    x0, y0, order = grid_geometry(Np, L, 2, 100)
    rng = np.random.default_rng(86)
    stack = rng.integers(0, 65535, (len(x0), 2, Np, Np)).astype(np.uint16)
    with fpm_amd.Solver(fpm_amd.Problem(Np, L, order, x0, y0, r, 5, 10, n_patch=2)) as s:
        s.upload(stack)
        np.testing.assert_array_equal(s.download_stack(), stack)


def test_np1024_fp16_scratch_vs_fp32_scratch():
    """fp16 spectrum storage puts the Np 1024 row / column scratch T in
    block-scaled fp16 too (one power-of-two scale per box row after the row
    IDFT, per column after the column pass); FPM_T32=1 keeps it fp32.  The two
    differ by fp16 rounding of T (2^-11 relative per element), well inside
    config 5's 1e-2."""
    L, r = 2048, 333
    x0, y0, order = grid_geometry(Np, L, 2, 100)
    stack = make_stack(Np, L, r, x0, y0, n_patch=2, seed=87)
    prob = fpm_amd.Problem(Np, L, order, x0, y0, r, 5, 10, n_patch=2, flags=fpm_amd.FLAG_SPEC_FP16)
    h = _run(prob, stack, 2)
    os.environ["FPM_T32"] = "1"
    try:
        f = _run(prob, stack, 2)
    finally:
        os.environ.pop("FPM_T32", None)
    for k in ("objF", "objCrop", "pupil"):
        for b in range(2):
            e = rel_l2(h[k][b], f[k][b])
            assert 0 < e < 2e-3, (k, b, e)


@pytest.mark.parametrize("fp16", [False, True], ids=["fp32", "fp16"])
def test_objcrop_l4096_six_step_equals_batched_transform(fp16):
    """objCrop at L 4096 (config 5): the six-step column IDFT (64 x 64, two
    passes of 128-byte row segments, general.hip c4k) then the in-place row
    IDFT, vs the batched transform rows-then-columns (FPM_NO_CROP4K=1): the
    same 2-D IDFT in a different order, so within rounding (1e-6 relative L2)."""
    L, r = 4096, 333
    x0, y0, order = grid_geometry(Np, L, 2, 600)
    stack = make_stack(Np, L, r, x0, y0, n_patch=1, seed=95)
    flags = fpm_amd.FLAG_SPEC_FP16 if fp16 else 0
    prob = fpm_amd.Problem(Np, L, order, x0, y0, r, 5, 10, n_patch=1, flags=flags)
    new = _run(prob, stack, 1)
    os.environ["FPM_NO_CROP4K"] = "1"
    try:
        old = _run(prob, stack, 1)
    finally:
        os.environ.pop("FPM_NO_CROP4K", None)
    np.testing.assert_array_equal(new["objF"][0], old["objF"][0])
    e = rel_l2(new["objCrop"][0], old["objCrop"][0])
    print(f"objCrop L 4096 six-step vs batched: rel L2 {e:.2e}")
    assert e < 1e-6, e
