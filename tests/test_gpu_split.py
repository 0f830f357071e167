"""Split mode of the Np 256 fused kernel (fpm_fused.hip): with
KS * n_patch <= CUs each patch runs on KS = 2 or 4 workgroups (one column part
each) that exchange their row-DFT partials once per LED through device-scope
flags (BASELINE config 4: 1024 patches over 8 GPUs = 128 per GPU; the
256-patch metric field strong-scaled over 4 / 8 GPUs = 64 / 32 per GPU).

  * KS = 2 adds the two partials in the same order as the one-workgroup kernel
    (F_0 + F_1), so the two agree bit for bit.
  * KS = 4 sums four quarter partials ((F_0 + F_1) + F_2) + F_3: the same
    arithmetic up to fp32 rounding (measured rel. L2 vs KS = 1 stated in the
    assertion), deterministic run to run, and checked against the fp64 oracle.
  * A handoff that times out (forced with fpm_debug_set_stall) fails fpm_run
    even when it happens in an earlier iteration of a multi-iteration run, and
    the context must be re-initialised.
"""
import os

import numpy as np
import pytest

import fpm_amd
from fpm_oracle import rel_l2
from tools.synth import grid_geometry, make_stack

pytestmark = pytest.mark.gpu


def _env(ks, dist):
    """Environment forcing ks workgroups per patch in split mode (dist False)
    or distributed mode (dist True); ks 1 = one workgroup per patch."""
    if ks == 1:
        return {"FPM_NO_SPLIT": "1", "FPM_NO_DIST": "1"}
    return {"FPM_DIST": str(ks)} if dist else {"FPM_SPLIT": str(ks), "FPM_NO_DIST": "1"}


def _solve(prob, stack, iters, ks, dist=False):
    env = _env(ks, dist)
    os.environ.update(env)
    try:
        with fpm_amd.Solver(prob) as s:
            info = s.info()
            want = fpm_amd.KERNEL_FUSED_NP256_DIST if dist else fpm_amd.KERNEL_FUSED_NP256
            assert info.fused_kernel == want
            s.upload(stack)
            s.init()
            s.run(iters)
            return info.wg_per_patch, s.download()
    finally:
        for k in env:
            os.environ.pop(k, None)


@pytest.mark.parametrize("r,nside,step,B,iters", [(33, 5, 20, 5, 2), (34, 3, 30, 9, 1), (10, 4, 24, 1, 3)],
                         ids=["r33_B5_it2", "r34_B9_it1", "r10_B1_it3"])
def test_split2_equals_one_workgroup_per_patch(r, nside, step, B, iters):
    Np, L = 256, 512
    x0, y0, order = grid_geometry(Np, L, nside, step)
    stack = make_stack(Np, L, r, x0, y0, n_patch=B, seed=5 + r)
    prob = fpm_amd.Problem(Np, L, order, x0, y0, r, 10, 3, n_patch=B, path=fpm_amd.PATH_FUSED)
    wg2, out2 = _solve(prob, stack, iters, 2)
    wg1, out1 = _solve(prob, stack, iters, 1)
    assert (wg2, wg1) == (2, 1)
    for k in ("objF", "objCrop", "pupil"):
        np.testing.assert_array_equal(out2[k], out1[k], err_msg=k)


@pytest.mark.parametrize("r,nside,step,B,iters", [(33, 5, 20, 5, 2), (34, 3, 30, 9, 1), (10, 4, 24, 1, 3)],
                         ids=["r33_B5_it2", "r34_B9_it1", "r10_B1_it3"])
def test_split4_matches_one_workgroup_and_oracle(r, nside, step, B, iters):
    import oracle_lib
    Np, L = 256, 512
    x0, y0, order = grid_geometry(Np, L, nside, step)
    stack = make_stack(Np, L, r, x0, y0, n_patch=B, seed=7 + r)
    prob = fpm_amd.Problem(Np, L, order, x0, y0, r, 10, 3, n_patch=B, path=fpm_amd.PATH_FUSED)
    wg4, out4 = _solve(prob, stack, iters, 4)
    wg4b, out4b = _solve(prob, stack, iters, 4)
    wg1, out1 = _solve(prob, stack, iters, 1)
    assert (wg4, wg4b, wg1) == (4, 4, 1)
    for k in ("objF", "objCrop", "pupil"):
        np.testing.assert_array_equal(out4[k], out4b[k], err_msg=k)      # deterministic
        for b in range(B):
            e = rel_l2(out4[k][b], out1[k][b])
            assert e < 2e-6, (k, b, e)                                     # fp32 summation order only
    tol = 1e-5 if iters == 1 else 5e-5
    for b in sorted({0, B - 1}):
        ref = oracle_lib.run_fpm(stack[:, b], order, x0, y0, Np, L, r, 10, 3, iters)
        for k in ("objF", "objCrop", "pupil"):
            assert rel_l2(out4[k][b], ref[k]) < tol, (k, b)


@pytest.mark.parametrize("ks,dist", [(2, False), (4, False), (2, True), (4, True), (8, True)],
                         ids=["split2", "split4", "dist2", "dist4", "dist8"])
def test_split_metric_geometry_many_handoffs(ks, dist):
    """293 LEDs of the metric geometry (one to three handoffs per LED) on 3
    patches: split / distributed vs one workgroup per patch, both finite and
    non-trivial."""
    from test_gpu_configs import _probe_geometry, _tiled_stack
    p, x0, y0 = _probe_geometry("geometry_dogStomach_metric.json")
    Np, L, r = p["np"], p["nlarge"], p["na_radius"]
    order = np.arange(len(x0))
    stack, _ = _tiled_stack(Np, L, r, x0, y0, 3, 3, seed=11)
    prob = fpm_amd.Problem(Np, L, order, x0, y0, r, p["delta1"], p["delta2"], n_patch=3, path=fpm_amd.PATH_FUSED)
    wgs, outs = _solve(prob, stack, 1, ks, dist)
    wg1, out1 = _solve(prob, stack, 1, 1)
    assert (wgs, wg1) == (ks, 1)
    assert np.isfinite(outs["objCrop"]).all()
    for k in ("objF", "objCrop", "pupil"):
        if ks == 2 and not dist:
            np.testing.assert_array_equal(outs[k], out1[k], err_msg=k)
        else:
            for b in range(3):
                assert rel_l2(outs[k][b], out1[k][b]) < 2e-6, (k, b)
    assert rel_l2(outs["objCrop"][0], outs["objCrop"][1]) > 1e-3  # patches differ


@pytest.mark.parametrize("ks", [2, 4, 8])
@pytest.mark.parametrize("r,nside,step,B,iters", [(33, 5, 20, 5, 2), (34, 3, 30, 3, 1), (10, 4, 24, 1, 3)],
                         ids=["r33_B5_it2", "r34_B3_it1", "r10_B1_it3"])
def test_distributed_matches_one_workgroup_and_oracle(r, nside, step, B, iters, ks):
    """Distributed mode (fused_dist.hip): rows, columns and the update
    partitioned over KS workgroups.  F is formed by one full-input row DFT
    instead of the sum of two half-input ones, so it agrees with the
    one-workgroup kernel to fp32 rounding (bound in the assertion); it is
    deterministic and matches the fp64 oracle."""
    import oracle_lib
    Np, L = 256, 512
    x0, y0, order = grid_geometry(Np, L, nside, step)
    stack = make_stack(Np, L, r, x0, y0, n_patch=B, seed=9 + r)
    prob = fpm_amd.Problem(Np, L, order, x0, y0, r, 10, 3, n_patch=B, path=fpm_amd.PATH_FUSED)
    wgd, outd = _solve(prob, stack, iters, ks, dist=True)
    wgd2, outd2 = _solve(prob, stack, iters, ks, dist=True)
    wg1, out1 = _solve(prob, stack, iters, 1)
    assert (wgd, wgd2, wg1) == (ks, ks, 1)
    for k in ("objF", "objCrop", "pupil"):
        np.testing.assert_array_equal(outd[k], outd2[k], err_msg=k)
        for b in range(B):
            e = rel_l2(outd[k][b], out1[k][b])
            assert e < 2e-6, (k, b, e)
    tol = 1e-5 if iters == 1 else 5e-5
    for b in sorted({0, B - 1}):
        ref = oracle_lib.run_fpm(stack[:, b], order, x0, y0, Np, L, r, 10, 3, iters)
        for k in ("objF", "objCrop", "pupil"):
            assert rel_l2(outd[k][b], ref[k]) < tol, (k, b)


@pytest.mark.parametrize("dist", [False, True], ids=["split4", "dist8"])
def test_handoff_timeout_is_reported_and_sticky(dist):
    """The last part stops publishing at LED 3 of the first iteration
    (fpm_debug_set_stall): its partners time out (~seconds), the abort word
    stays set through the second launch of fpm_run(2), the run fails with
    FPM_ERR_DEVICE, and the context needs fpm_init again (after which a clean
    run succeeds).  Split mode (4 parts) and the distributed mode (8 parts,
    three handoffs per LED) both."""
    Np, L, r = 256, 512, 10
    x0, y0, order = grid_geometry(Np, L, 3, 24)
    stack = make_stack(Np, L, r, x0, y0, n_patch=1, seed=3)
    prob = fpm_amd.Problem(Np, L, order, x0, y0, r, 10, 3, n_patch=1, path=fpm_amd.PATH_FUSED)
    env = {"FPM_DIST": "8"} if dist else {"FPM_NO_DIST": "1"}
    os.environ.update(env)
    try:
        s = fpm_amd.Solver(prob)
    finally:
        for k in env:
            os.environ.pop(k, None)
    with s:
        info = s.info()
        assert info.wg_per_patch == (8 if dist else 4)
        assert info.fused_kernel == (fpm_amd.KERNEL_FUSED_NP256_DIST if dist else fpm_amd.KERNEL_FUSED_NP256)
        s.upload(stack)
        s.init()
        s.debug_set_stall(3)
        with pytest.raises(fpm_amd.FpmError) as e:
            s.run(2)
        s.debug_set_stall(-1)
        assert e.value.code == fpm_amd.FPM_ERR_DEVICE
        assert "timed out" in str(e.value)
        with pytest.raises(fpm_amd.FpmError) as e2:  # state is undefined until re-initialised
            s.run(1)
        assert e2.value.code == fpm_amd.FPM_ERR_STATE
        s.init()
        s.run(1)
        out = s.download()
    assert np.isfinite(out["objCrop"]).all()
