"""The large-radius fused Np 256 kernel (csrc/fused_large.hip: one
1024-thread workgroup per patch, one launch per iteration, the row-transform
scratch in global memory) for 34 < r < 128 -- the dataset_mono geometry at
cropSizeX 256 has r 84 -- vs the general path's register kernels
(csrc/np256.hip, PATH_GENERAL) and vs the C++ fp64 oracle (GPU only).  The
full-size dataset_mono case (64 patches, 193 LEDs, 2 iterations) is
tests/test_gpu_configs.py::test_config2_geometry_at_np256_r84_64_patches.

Tolerance: relative L2 <= 1e-5 against the oracle after 1 iteration (as every
fp32 path), <= 1e-5 between the two GPU implementations after 2 iterations
(the same transforms in the same order; the exact max|objF| from the same
tile maxima).
"""
import numpy as np
import pytest

import fpm_amd
from fpm_oracle import rel_l2
from tools.synth import grid_geometry, make_stack

pytestmark = pytest.mark.gpu

Np = 256


def _problem(L, r, B, x0, y0, order, path=fpm_amd.PATH_AUTO):
    return fpm_amd.Problem(Np, L, order, x0, y0, r, 5, 10, n_patch=B, path=path)


@pytest.mark.parametrize("L,r,B", [(768, 84, 2), (768, 35, 3), (1024, 84, 8), (256, 127, 2)],
                         ids=["r84", "r35_3patches", "r84_8patches", "r127_edges"])
def test_fused_large_equals_general_register_path(L, r, B):
    if L == Np:  # one LED: the crop covers the whole spectrum (crop 0, 0)
        x0, y0, order = np.array([0, 0]), np.array([0, 0]), [0, 1]
    else:
        x0, y0, order = grid_geometry(Np, L, 3 if L > 768 else 2, 60)
    stack = make_stack(Np, L, r, x0, y0, n_patch=B, seed=360 + r + B)
    prob = _problem(L, r, B, x0, y0, order)
    with fpm_amd.Solver(prob) as s:
        info = s.info()
        assert info.path == fpm_amd.PATH_FUSED and info.fused_kernel == fpm_amd.KERNEL_FUSED_NP256_LARGE
        assert info.threads_per_wg == 1024 and info.wg_per_patch == 1
    fused = fpm_amd.run_fpm(prob, stack, 2)
    gen = fpm_amd.run_fpm(_problem(L, r, B, x0, y0, order, fpm_amd.PATH_GENERAL), stack, 2)
    for k in ("objF", "objCrop", "pupil"):
        for b in range(B):
            e = rel_l2(fused[k][b], gen[k][b])
            assert e < 1e-5, (k, b, e)


def test_fused_large_vs_oracle():
    import oracle_lib
    L, r = 768, 84
    x0, y0, order = grid_geometry(Np, L, 3, 50)
    stack = make_stack(Np, L, r, x0, y0, n_patch=1, seed=365)
    out = fpm_amd.run_fpm(_problem(L, r, 1, x0, y0, order), stack, 1)
    ref = oracle_lib.run_fpm(stack[:, 0], order, x0, y0, Np, L, r, 5, 10, 1)
    for k in ("objF", "objCrop", "pupil"):
        e = rel_l2(out[k][0], ref[k])
        print(f"fused large r 84 {k} rel L2 {e:.2e}")
        assert e < 1e-5, k


def test_fused_large_three_iterations_vs_oracle():
    """Three iterations: the kernel carries max|P| and the tile maxima across
    launches (pmax, tmax), the pupil commit of every LED inside the launch."""
    import oracle_lib
    L, r = 1024, 84
    x0, y0, order = grid_geometry(Np, L, 3, 70)
    stack = make_stack(Np, L, r, x0, y0, n_patch=1, seed=366)
    out = fpm_amd.run_fpm(_problem(L, r, 1, x0, y0, order), stack, 3)
    ref = oracle_lib.run_fpm(stack[:, 0], order, x0, y0, Np, L, r, 5, 10, 3)
    for k in ("objF", "objCrop", "pupil"):
        e = rel_l2(out[k][0], ref[k])
        print(f"fused large r 84, 3 iterations {k} rel L2 {e:.2e}")
        assert e < 5e-5, k
