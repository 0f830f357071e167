"""Np 90 kernel distributed over 2 / 4 workgroups per patch
(csrc/fused_s90d.hip, FPM_S90D=2/4) -- the partition of the Np 256
distributed kernel (fused_dist.hip) on fused_s90.hip's register transforms,
for BASELINE config 2 (64 patches would leave 192 of the 256 CUs idle with one
workgroup per patch).  Every element is computed by the same operations as in
the one-workgroup kernel (the T image's round trip through L2 is exact), so
the outputs must be BIT-IDENTICAL to it; one case is also checked against the
C++ fp64 oracle (tolerances as tests/test_gpu_fused_s90.py)."""
import os

import numpy as np
import pytest

import fpm_amd
from fpm_oracle import rel_l2
from tools.synth import grid_geometry, make_stack

pytestmark = pytest.mark.gpu


def _solve(prob, stack, iters, ks):
    env = {"FPM_S90D": str(ks)} if ks > 1 else {}
    os.environ.update(env)
    try:
        s = fpm_amd.Solver(prob)
    finally:
        for k in env:
            os.environ.pop(k, None)
    with s:
        info = s.info()
        assert info.fused_kernel == fpm_amd.KERNEL_FUSED_NP90
        assert info.wg_per_patch == ks
        s.upload(stack)
        s.init()
        s.run(iters)
        return s.download()


CASES = [  # L, r, n_side, step, iters, B
    (360, 30, 4, 22, 2, 3),   # configs 1/2 optics on a synthetic grid
    (360, 12, 3, 30, 1, 1),
    (270, 44, 3, 20, 2, 2),   # the largest radius (2r + 1 = 89 box rows)
    (180, 3, 2, 10, 3, 9),    # more patches than one round of eight
]


@pytest.mark.parametrize("ks", [2, 4])
@pytest.mark.parametrize("L,r,nside,step,iters,B", CASES, ids=[f"r{c[1]}_it{c[4]}_B{c[5]}" for c in CASES])
def test_s90d_bit_identical_to_one_workgroup(L, r, nside, step, iters, B, ks):
    Np = 90
    x0, y0, order = grid_geometry(Np, L, nside, step)
    stack = make_stack(Np, L, r, x0, y0, n_patch=B, seed=191 + r)
    prob = fpm_amd.Problem(Np, L, order, x0, y0, r, 5, 10, n_patch=B, path=fpm_amd.PATH_FUSED)
    one = _solve(prob, stack, iters, 1)
    dist = _solve(prob, stack, iters, ks)
    for k in ("objF", "objCrop", "pupil"):
        assert np.array_equal(one[k], dist[k]), (k, float(np.abs(one[k] - dist[k]).max()))


def test_s90d_config2_batch_vs_oracle():
    """64 patches (config 2's batch: 256 co-resident workgroups at 4 parts),
    1 iteration; first / middle / last patch against the fp64 oracle and the
    whole batch bit-identical to one workgroup per patch."""
    import oracle_lib
    Np, L, r, B = 90, 360, 30, 64
    x0, y0, order = grid_geometry(Np, L, 5, 20)
    stack = make_stack(Np, L, r, x0, y0, n_patch=B, seed=964)
    prob = fpm_amd.Problem(Np, L, order, x0, y0, r, 5, 10, n_patch=B, path=fpm_amd.PATH_FUSED)
    dist = _solve(prob, stack, 1, 4)
    one = _solve(prob, stack, 1, 1)
    for k in ("objF", "objCrop", "pupil"):
        assert np.array_equal(one[k], dist[k]), k
    for b in (0, B // 2, B - 1):
        ref = oracle_lib.run_fpm(stack[:, b], order, x0, y0, Np, L, r, 5, 10, 1)
        for k in ("objCrop", "pupil"):
            e = rel_l2(dist[k][b], ref[k])
            assert e < 1e-5, (k, b, e)


def test_s90d_handoff_timeout_is_reported_and_sticky():
    """The last part stops publishing at LED 3 (fpm_debug_set_stall): the
    partners time out, the run fails with FPM_ERR_DEVICE, the context needs
    fpm_init again, and a clean run then succeeds."""
    Np, L, r = 90, 360, 12
    x0, y0, order = grid_geometry(Np, L, 3, 30)
    stack = make_stack(Np, L, r, x0, y0, n_patch=1, seed=5)
    prob = fpm_amd.Problem(Np, L, order, x0, y0, r, 5, 10, n_patch=1, path=fpm_amd.PATH_FUSED)
    os.environ["FPM_S90D"] = "4"
    try:
        s = fpm_amd.Solver(prob)
    finally:
        os.environ.pop("FPM_S90D", None)
    with s:
        assert s.info().wg_per_patch == 4
        s.upload(stack)
        s.init()
        s.debug_set_stall(3)
        with pytest.raises(fpm_amd.FpmError) as e:
            s.run(2)
        s.debug_set_stall(-1)
        assert e.value.code == fpm_amd.FPM_ERR_DEVICE
        assert "timed out" in str(e.value)
        with pytest.raises(fpm_amd.FpmError) as e2:
            s.run(1)
        assert e2.value.code == fpm_amd.FPM_ERR_STATE
        s.init()
        s.run(1)
        out = s.download()
    assert np.isfinite(out["objCrop"]).all()
