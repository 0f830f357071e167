"""Patch groups of the general path (api.cpp launch_general_iteration): the
context's patches split into G groups whose per-LED launches run on G
concurrent streams (FPM_PATCH_GROUPS; two by default for the Np 1024
kernels).  Patches are independent (fpmMain.cpp:274-498 runs runFPM per
patch), so every G must give the same bits as G = 1, with and without the
captured iteration graph, and match the fp64 oracle."""
import os

import numpy as np
import pytest

import fpm_amd
from fpm_oracle import rel_l2
from tools.synth import grid_geometry, make_stack

pytestmark = pytest.mark.gpu


def _solve(prob, stack, iters, groups, graph=True):
    env = {"FPM_PATCH_GROUPS": str(groups)}
    if not graph:
        env["FPM_NO_GRAPH"] = "1"
    os.environ.update(env)
    try:
        with fpm_amd.Solver(prob) as s:
            assert s.info().path == fpm_amd.PATH_GENERAL
            s.upload(stack)
            s.init()
            s.run(iters)
            return s.download()
    finally:
        for k in env:
            os.environ.pop(k, None)


@pytest.mark.parametrize("np_,L,r,nside,step,B,flags", [
    (1024, 2048, 100, 3, 60, 3, fpm_amd.FLAG_SPEC_FP16),   # the Np 1024 register kernels (config 5 path)
    (1024, 2048, 100, 2, 80, 2, 0),
    (64, 192, 10, 5, 10, 5, 0),                             # the tiled general kernels
], ids=["np1024_fp16_B3", "np1024_B2", "np64_B5"])
def test_patch_groups_bit_identical(np_, L, r, nside, step, B, flags):
    x0, y0, order = grid_geometry(np_, L, nside, step)
    stack = make_stack(np_, L, r, x0, y0, n_patch=B, seed=21 + B)
    prob = fpm_amd.Problem(np_, L, order, x0, y0, r, 5, 10, n_patch=B, path=fpm_amd.PATH_GENERAL, flags=flags)
    ref = _solve(prob, stack, 2, 1)
    for groups, graph in ((2, True), (2, False), (B, True)):
        got = _solve(prob, stack, 2, groups, graph)
        for k in ("objF", "objCrop", "pupil"):
            np.testing.assert_array_equal(got[k], ref[k], err_msg=f"{k} groups={groups} graph={graph}")
    assert rel_l2(ref["objCrop"][0], ref["objCrop"][B - 1]) > 1e-3  # patches differ


def test_patch_groups_np1024_vs_oracle():
    import oracle_lib
    Np, L, r, B = 1024, 2048, 100, 2
    x0, y0, order = grid_geometry(Np, L, 2, 80)
    stack = make_stack(Np, L, r, x0, y0, n_patch=B, seed=33)
    prob = fpm_amd.Problem(Np, L, order, x0, y0, r, 5, 10, n_patch=B, path=fpm_amd.PATH_GENERAL)
    out = _solve(prob, stack, 1, 2)
    for b in range(B):
        ref = oracle_lib.run_fpm(stack[:, b], order, x0, y0, Np, L, r, 5, 10, 1)
        for k in ("objCrop", "objF", "pupil"):
            assert rel_l2(out[k][b], ref[k]) < 1e-5, (k, b)
