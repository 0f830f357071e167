"""Split mode of the Np 256 fused kernel (fpm_fused.hip): with n_patch <= CUs/2
each patch runs on two workgroups (one column half each) that hand the row-DFT
partials and the updated pupil to each other through device-scope flags
(BASELINE config 4: 1024 patches over 8 GPUs = 128 per GPU).  The split path
adds the two halves' partials in the same order as the one-workgroup path, so
the two must agree bit for bit; parity with the oracle is covered by every
small-batch fused test (tests/test_gpu_parity.py runs n_patch 2, i.e. split).
"""
import os

import numpy as np
import pytest

import fpm_amd
from fpm_oracle import rel_l2
from tools.synth import grid_geometry, make_stack

pytestmark = pytest.mark.gpu


def _solve(prob, stack, iters, no_split):
    if no_split:
        os.environ["FPM_NO_SPLIT"] = "1"
    try:
        with fpm_amd.Solver(prob) as s:
            info = s.info()
            s.upload(stack)
            s.init()
            s.run(iters)
            return info.wg_per_patch, s.download()
    finally:
        os.environ.pop("FPM_NO_SPLIT", None)


@pytest.mark.parametrize("r,nside,step,B,iters", [(33, 5, 20, 5, 2), (34, 3, 30, 9, 1), (10, 4, 24, 1, 3)],
                         ids=["r33_B5_it2", "r34_B9_it1", "r10_B1_it3"])
def test_split_equals_one_workgroup_per_patch(r, nside, step, B, iters):
    Np, L = 256, 512
    x0, y0, order = grid_geometry(Np, L, nside, step)
    stack = make_stack(Np, L, r, x0, y0, n_patch=B, seed=5 + r)
    prob = fpm_amd.Problem(Np, L, order, x0, y0, r, 10, 3, n_patch=B, path=fpm_amd.PATH_FUSED)
    wg2, out2 = _solve(prob, stack, iters, no_split=False)
    wg1, out1 = _solve(prob, stack, iters, no_split=True)
    assert (wg2, wg1) == (2, 1)
    for k in ("objF", "objCrop", "pupil"):
        np.testing.assert_array_equal(out2[k], out1[k], err_msg=k)


def test_split_metric_geometry_many_handoffs():
    """293 LEDs of the metric geometry (586 handoffs per iteration) on 3 patches:
    split vs one workgroup per patch, and both finite and non-trivial."""
    from test_gpu_configs import _probe_geometry, _tiled_stack
    p, x0, y0 = _probe_geometry("geometry_dogStomach_metric.json")
    Np, L, r = p["np"], p["nlarge"], p["na_radius"]
    order = np.arange(len(x0))
    stack, _ = _tiled_stack(Np, L, r, x0, y0, 3, 3, seed=11)
    prob = fpm_amd.Problem(Np, L, order, x0, y0, r, p["delta1"], p["delta2"], n_patch=3, path=fpm_amd.PATH_FUSED)
    wg2, out2 = _solve(prob, stack, 1, no_split=False)
    wg1, out1 = _solve(prob, stack, 1, no_split=True)
    assert (wg2, wg1) == (2, 1)
    assert np.isfinite(out2["objCrop"]).all()
    for k in ("objF", "objCrop", "pupil"):
        np.testing.assert_array_equal(out2[k], out1[k], err_msg=k)
    assert rel_l2(out2["objCrop"][0], out2["objCrop"][1]) > 1e-3  # patches differ
